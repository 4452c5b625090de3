// mtg_capi.hip -- the C ABI (include/mtg.h): contexts, staging, launches.
// Never aborts, never throws across the boundary; errors are return codes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <pthread.h>
#include <sched.h>

#include <cctype>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "mtg.h"
#include "mtg_internal.h"

// A persistent host thread of a context that runs one job at a time for the caller (the pipelined
// solve's D2H issuer): created on first use and kept, instead of a std::thread per call (~50-100 us of
// thread creation per host-array solve), and bound to the CPUs of the GPU's NUMA node where the
// process may run there (the pageable-copy staging and completion waits then stay node-local).
struct CtxWorker {
  std::thread th;
  std::mutex m;
  std::condition_variable cv;
  std::function<void()> job;
  bool has_job = false, quit = false;
  ~CtxWorker() {
    if (!th.joinable()) return;
    {
      std::lock_guard<std::mutex> g(m);
      quit = true;
    }
    cv.notify_all();
    th.join();
  }
  // start the thread (once); false if no thread can be created
  bool start(const cpu_set_t* affinity) {
    if (th.joinable()) return true;
    try {
      th = std::thread([this] {
        std::unique_lock<std::mutex> l(m);
        for (;;) {
          cv.wait(l, [this] { return has_job || quit; });
          if (quit) return;
          std::function<void()> j = std::move(job);
          l.unlock();
          j();
          l.lock();
          has_job = false;
          cv.notify_all();
        }
      });
    } catch (...) {
      return false;
    }
    if (affinity) (void)pthread_setaffinity_np(th.native_handle(), sizeof(cpu_set_t), affinity);
    return true;
  }
  void post(std::function<void()> j) {
    std::lock_guard<std::mutex> g(m);
    job = std::move(j);
    has_job = true;
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> l(m);
    cv.wait(l, [this] { return !has_job; });
  }
};

struct mtg_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  void* staging = nullptr;
  size_t staging_bytes = 0;
  void* workspace = nullptr;
  size_t workspace_bytes = 0;
  void* pinned = nullptr;  // host mirror of the staging layout for small calls (hipHostMalloc)
  size_t pinned_bytes = 0;
  // ring of (start, stop) events around kernel launches; launches counts recorded launches
  std::vector<hipEvent_t> ev_start, ev_stop;
  int64_t launches = 0;
  std::string last_error;
  std::mutex mu;
  int inject_rc = 0;  // mtg_debug_fail_next_solve: the next solve's return code (0: none)
  // Pipelined host-pointer solves (run_solve_pipelined): kPipeSlots chunks in flight, each with its
  // own kernel stream and device buffers; all H2D copies go through one stream and all D2H copies
  // through another (one copy queue per direction).
  static constexpr int kPipeSlots = 4;
  struct PipeSlot {
    hipStream_t stream = nullptr;  // the chunk's kernel
    hipEvent_t in_done = nullptr;  // its H2D copies landed (recorded on pipe_h2d)
    hipEvent_t k_done = nullptr;   // its kernel finished (recorded on stream)
    hipEvent_t done = nullptr;     // its D2H copies landed (recorded on pipe_d2h)
    void* dev = nullptr;  // device inputs + outputs of one chunk
    size_t dev_bytes = 0;
  } pipe[kPipeSlots];
  hipStream_t pipe_h2d = nullptr, pipe_d2h = nullptr;
  hipEvent_t pipe_start = nullptr;
  CtxWorker d2h_worker;
};

namespace mtg {
PendingEvents& pending_events() {
  static thread_local PendingEvents pe;
  return pe;
}
}  // namespace mtg

namespace {

int set_hip_error(mtg_ctx* ctx, hipError_t e, const char* what) {
  if (ctx) {
    char buf[256];
    snprintf(buf, sizeof(buf), "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    ctx->last_error = buf;
  }
  return e == hipErrorOutOfMemory ? MTG_ERR_OUT_OF_MEMORY : MTG_ERR_HIP;
}

int set_error(mtg_ctx* ctx, int code, const char* what) {
  if (ctx) ctx->last_error = what;
  return code;
}

#define MTG_HIP_TRY(ctx, expr)                          \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return set_hip_error(ctx, e_, #expr); \
  } while (0)

size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// host-pointer calls whose staged arrays fit this size go through one pinned buffer
constexpr size_t kPinnedMax = 1u << 20;

hipError_t ensure(void** buf, size_t* have, size_t need) {
  if (*have >= need) return hipSuccess;
  if (*buf) {
    hipError_t e = hipFree(*buf);
    if (e != hipSuccess) return e;
    *buf = nullptr;
    *have = 0;
  }
  hipError_t e = hipMalloc(buf, need);
  if (e == hipSuccess) *have = need;
  return e;
}

// Timed region around one launch.  single: the call launches exactly one kernel through
// mtg::launch_kernel, which carries the event pair in its dispatch packet; otherwise (the split
// path's two kernels) the events are recorded as stream markers around the launches.
hipError_t time_begin(mtg_ctx* ctx, bool single = true) {
  mtg::PendingEvents& pe = mtg::pending_events();
  pe = mtg::PendingEvents{};
  if (ctx->ev_start.empty()) return hipSuccess;  // timing disabled (mtg_enable_timing(ctx, 0))
  const size_t slot = (size_t)(ctx->launches % (int64_t)ctx->ev_start.size());
  if (single) {
    pe.start = ctx->ev_start[slot];
    pe.stop = ctx->ev_stop[slot];
    return hipSuccess;
  }
  return hipEventRecord(ctx->ev_start[slot], ctx->stream);
}

hipError_t time_end(mtg_ctx* ctx) {
  if (ctx->ev_start.empty()) return hipSuccess;
  const size_t slot = (size_t)(ctx->launches % (int64_t)ctx->ev_start.size());
  mtg::PendingEvents& pe = mtg::pending_events();
  hipError_t e = hipSuccess;
  if (pe.start) {
    if (!pe.used) {  // nothing was launched (e.g. an empty batch): an empty interval
      e = hipEventRecord(pe.start, ctx->stream);
      if (e == hipSuccess) e = hipEventRecord(pe.stop, ctx->stream);
    }
    pe = mtg::PendingEvents{};
  } else {
    e = hipEventRecord(ctx->ev_stop[slot], ctx->stream);
  }
  if (e == hipSuccess) ctx->launches++;
  return e;
}

void destroy_events(mtg_ctx* ctx) {
  for (hipEvent_t e : ctx->ev_start) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->ev_stop) (void)hipEventDestroy(e);
  ctx->ev_start.clear();
  ctx->ev_stop.clear();
  ctx->launches = 0;
}

hipError_t create_events(mtg_ctx* ctx, int ring) {
  destroy_events(ctx);
  for (int i = 0; i < ring; ++i) {
    hipEvent_t a = nullptr, b = nullptr;
    hipError_t e = hipEventCreate(&a);
    if (e == hipSuccess) e = hipEventCreate(&b);
    if (e != hipSuccess) {
      if (a) (void)hipEventDestroy(a);
      return e;
    }
    ctx->ev_start.push_back(a);
    ctx->ev_stop.push_back(b);
  }
  return hipSuccess;
}

int check_shape(mtg_ctx* ctx, int N, int D, int K, int r, int64_t batch) {
  if (!ctx) return MTG_ERR_INVALID_ARGUMENT;
  if (N < 2 || N > 12 || (N % 2)) return set_error(ctx, MTG_ERR_UNSUPPORTED_N, "N must be even and in [2, 12]");
  if (r < 0 || r > N / 2 - 1)
    return set_error(ctx, MTG_ERR_BAD_DERIVATIVE, "derivative_to_optimize must be in [0, N/2-1]");
  if (K < 1 || D < 1 || batch < 0) return set_error(ctx, MTG_ERR_SIZE_MISMATCH, "need K >= 1, D >= 1, batch >= 0");
  int lg, tpb;
  size_t lds;
  if (!mtg::solve_geometry(N, D, K, &lg, &lds, &tpb))
    return set_error(ctx, MTG_ERR_TOO_LARGE, "per-trajectory working set exceeds LDS (reduce K or D)");
  return MTG_OK;
}

// MTG_HOST_WAIT=block: the pipeline's D2H thread sleeps on its chunk events (hipEventBlockingSync)
// instead of spinning on them (the runtime's default).  For measuring the host work of several
// concurrent pipelines (scripts/multi_host_cost.py): spinning waits make every waiting thread count
// as a busy core.  Read once per process.
bool host_wait_blocking() {
  static const bool b = [] {
    const char* v = getenv("MTG_HOST_WAIT");
    return v && strcmp(v, "block") == 0;
  }();
  return b;
}

hipError_t ensure_pipe(mtg_ctx* ctx) {
  if (ctx->pipe_start) return hipSuccess;
  const unsigned done_flags = hipEventDisableTiming | (host_wait_blocking() ? hipEventBlockingSync : 0u);
  for (auto& s : ctx->pipe) {
    hipError_t e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.in_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.k_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.done, done_flags);
    if (e != hipSuccess) return e;
  }
  hipError_t e = hipStreamCreateWithFlags(&ctx->pipe_h2d, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->pipe_d2h, hipStreamNonBlocking);
  if (e != hipSuccess) return e;
  return hipEventCreateWithFlags(&ctx->pipe_start, hipEventDisableTiming);
}

void destroy_pipe(mtg_ctx* ctx) {
  for (hipStream_t* q : {&ctx->pipe_h2d, &ctx->pipe_d2h}) {
    if (*q) (void)hipStreamSynchronize(*q);
  }
  for (auto& s : ctx->pipe) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.dev) (void)hipFree(s.dev);
    for (hipEvent_t ev : {s.in_done, s.k_done, s.done})
      if (ev) (void)hipEventDestroy(ev);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = mtg_ctx::PipeSlot{};
  }
  for (hipStream_t* q : {&ctx->pipe_h2d, &ctx->pipe_d2h}) {
    if (*q) (void)hipStreamDestroy(*q);
    *q = nullptr;
  }
  if (ctx->pipe_start) (void)hipEventDestroy(ctx->pipe_start);
  ctx->pipe_start = nullptr;
}

// The CPUs of the device's NUMA node that this process may run on (sysfs: the PCI device's numa_node
// and the node's cpulist), or nullptr when unknown, empty, or MTG_NO_NUMA_BIND is set.
const cpu_set_t* gpu_node_cpus(int device) {
  constexpr int kDevs = 64;
  static std::mutex mu;
  static cpu_set_t sets[kDevs];
  static bool known[kDevs] = {};
  if (device < 0 || device >= kDevs) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (known[device]) return CPU_COUNT(&sets[device]) ? &sets[device] : nullptr;
  cpu_set_t& set = sets[device];
  CPU_ZERO(&set);
  char bus[64] = {0};
  const char* off = getenv("MTG_NO_NUMA_BIND");
  if (!(off && *off && *off != '0') && hipDeviceGetPCIBusId(bus, sizeof(bus), device) == hipSuccess) {
    for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
    char path[160];
    snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
    int node = -1;
    if (FILE* f = fopen(path, "r")) {
      if (fscanf(f, "%d", &node) != 1) node = -1;
      fclose(f);
    }
    cpu_set_t allowed;
    CPU_ZERO(&allowed);
    if (node >= 0 && sched_getaffinity(0, sizeof(allowed), &allowed) == 0) {
      snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
      if (FILE* f = fopen(path, "r")) {
        int a = 0, b = 0;
        char sep = 0;
        while (fscanf(f, "%d", &a) == 1) {
          b = a;
          if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
            if (fscanf(f, "%d", &b) != 1) b = a;
            if (fscanf(f, "%c", &sep) != 1) sep = 0;
          }
          for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &allowed)) CPU_SET(c, &set);
          if (sep != ',') break;
        }
        fclose(f);
      }
    }
  }
  known[device] = true;
  return CPU_COUNT(&set) ? &set : nullptr;
}

// host-pointer solves above this size go through the chunked pipeline
constexpr size_t kPipelineMinBytes = 8u << 20;
// returned by run_solve_pipelined when it could not start its D2H thread (nothing was issued)
constexpr int kPipelineUnavailable = 1;

// Host-pointer batch solve as a pipeline of chunks (the reference's equivalent is a
// loop of single solves, src/polynomial_timing_evaluation.cpp:119-126).  Each of kPipeSlots slots
// has its own kernel stream and device buffers.  This thread issues, per chunk, the H2D copies (on
// the context's one H2D stream) and the kernel (on the slot's stream, after the copies); a second
// host thread issues the chunk's D2H copies (on the one D2H stream, after the kernel) and retires
// it.  So the H2D of chunk c+1 runs on one DMA direction while the D2H of chunk c runs on the other
// (PCIe is full duplex: ~57 GB/s each way on MI355X, 97 GB/s both, scripts/pcie_bw.py), whether the
// caller's arrays are pinned (asynchronous copies) or pageable (the runtime's own staging, which
// blocks the issuing thread -- hence two threads).  One stream per copy direction: with the copies
// on the four slot streams, a pinned caller's copies of both directions were spread over the
// runtime's copy queues and the call ran in two modes (config 2, B = 125000: 7.0 or ~10-13 ms per
// call, median 9.8; pageable 6.6 ms).  A slot is reused only after its previous chunk's D2H completed.
int run_solve_pipelined(mtg_ctx* ctx, int N, int D, int K, int r, int64_t batch, const double* values,
                        const uint8_t* mask, const double* times, double* coeffs, double* free_out,
                        int32_t* n_free_out, double* cost_out, int32_t* status, unsigned kflags) {
  constexpr int S = mtg_ctx::kPipeSlots;
  const int V = K + 1, h = N / 2;
  // per-trajectory bytes of each array
  const size_t s_vals = sizeof(double) * (size_t)V * h * D, s_mask = (size_t)V, s_times = sizeof(double) * K;
  const size_t s_coef = coeffs ? sizeof(double) * (size_t)K * D * N : 0;
  const size_t s_free = free_out ? sizeof(double) * D * V * h : 0;
  const size_t s_nfree = n_free_out ? sizeof(int32_t) : 0, s_cost = cost_out ? sizeof(double) : 0;
  const size_t s_status = status ? sizeof(int32_t) : 0;
  const size_t per_traj = s_vals + s_mask + s_times + s_coef + s_free + s_nfree + s_cost + s_status;
  // a quarter of the batch per chunk (the pipeline fills and drains in a quarter of the run), at
  // most ~32 MB of traffic per chunk (per-chunk issue costs stay below ~5%)
  int64_t chunk = std::min<int64_t>((batch + 3) / 4, (int64_t)((32u << 20) / per_traj));
  chunk = (std::max<int64_t>(chunk, 1024) + 63) / 64 * 64;
  const int64_t n_chunks = (batch + chunk - 1) / chunk;
  size_t off = 0;  // one slot's device layout, 256-B aligned sub-buffers
  const size_t o_vals = off; off = align_up(off + s_vals * chunk);
  const size_t o_mask = off; off = align_up(off + s_mask * chunk);
  const size_t o_times = off; off = align_up(off + s_times * chunk);
  const size_t o_coef = off; off = align_up(off + s_coef * chunk);
  const size_t o_free = off; off = align_up(off + s_free * chunk);
  const size_t o_nfree = off; off = align_up(off + s_nfree * chunk);
  const size_t o_cost = off; off = align_up(off + s_cost * chunk);
  const size_t o_status = off; off = align_up(off + s_status * chunk);
  // the long-chain DL kernel's workspace, per slot (the slots' kernels may run at once)
  const unsigned ksel = kflags & (MTG_FLAG_GENERAL_KERNEL | MTG_FLAG_DL_KERNEL | MTG_FLAG_COLUMN_KERNEL);
  const size_t s_work = mtg::solve_kernel(N, D, K, ksel, r, chunk) == MTG_KERNEL_DLX
                            ? mtg::dlx_workspace_bytes(N, D, K, chunk) : 0;
  const size_t o_work = off; off = align_up(off + s_work);
  MTG_HIP_TRY(ctx, ensure_pipe(ctx));
  for (auto& s : ctx->pipe) MTG_HIP_TRY(ctx, ensure(&s.dev, &s.dev_bytes, off));

  std::mutex m;
  std::condition_variable cv;
  int64_t launched = 0, retired = 0;  // chunks whose kernel is queued / whose outputs have landed
  hipError_t err = hipSuccess;
  const char* err_what = "";
  auto fail = [&](hipError_t e, const char* what) {
    std::lock_guard<std::mutex> g(m);
    if (err == hipSuccess) err = e, err_what = what;
    cv.notify_all();
  };
  // D2H issuer: chunk c's outputs into the caller's arrays, on the chunk's slot stream (ordered after
  // its kernel), then wait for them and retire the chunk
  auto d2h_body = [&] {
    hipError_t e = hipSetDevice(ctx->device);
    if (e != hipSuccess) return fail(e, "hipSetDevice");
    for (int64_t c = 0; c < n_chunks; ++c) {
      {
        std::unique_lock<std::mutex> l(m);
        cv.wait(l, [&] { return launched > c || err != hipSuccess; });
        if (err != hipSuccess) return;
      }
      mtg_ctx::PipeSlot& s = ctx->pipe[c % S];
      const int64_t b0 = c * chunk, nb = std::min<int64_t>(chunk, batch - b0);
      const char* dp = static_cast<const char*>(s.dev);
      auto copy = [&](void* user, size_t o, size_t sz) -> hipError_t {
        return sz ? hipMemcpyAsync((char*)user + b0 * sz, dp + o, nb * sz, hipMemcpyDeviceToHost, ctx->pipe_d2h)
                  : hipSuccess;
      };
      e = hipStreamWaitEvent(ctx->pipe_d2h, s.k_done, 0);
      if (e == hipSuccess) e = copy(coeffs, o_coef, s_coef);
      if (e == hipSuccess) e = copy(free_out, o_free, s_free);
      if (e == hipSuccess) e = copy(n_free_out, o_nfree, s_nfree);
      if (e == hipSuccess) e = copy(cost_out, o_cost, s_cost);
      if (e == hipSuccess) e = copy(status, o_status, s_status);
      if (e == hipSuccess) e = hipEventRecord(s.done, ctx->pipe_d2h);
      // retire the previous chunk (its copies queued before this one's, so the DMA engine never
      // idles between chunks while this thread waits), and the last one at the end
      if (e == hipSuccess && c > 0) e = hipEventSynchronize(ctx->pipe[(c - 1) % S].done);
      if (e == hipSuccess && c + 1 == n_chunks) e = hipEventSynchronize(s.done);
      if (e != hipSuccess) return fail(e, "pipelined D2H");
      std::lock_guard<std::mutex> g(m);
      retired = c + 1 == n_chunks ? n_chunks : c;
      cv.notify_all();
    }
  };
  if (!ctx->d2h_worker.start(gpu_node_cpus(ctx->device)))
    return kPipelineUnavailable;  // no thread (std::system_error): nothing was issued, the caller stages
  ctx->d2h_worker.post(d2h_body);
  {
    // the pipeline's whole span (every chunk's H2D, kernel and D2H) is this call's timed interval;
    // the slot streams start after whatever the caller queued on the context's stream
    hipError_t e = time_begin(ctx, false);
    if (e == hipSuccess) e = hipEventRecord(ctx->pipe_start, ctx->stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(ctx->pipe_h2d, ctx->pipe_start, 0);
    if (e != hipSuccess) fail(e, "pipeline start");
  }
  // H2D + kernel issuer (this thread)
  for (int64_t c = 0; c < n_chunks; ++c) {
    {
      std::unique_lock<std::mutex> l(m);  // the slot's previous chunk must have landed
      cv.wait(l, [&] { return retired >= c - S + 1 || err != hipSuccess; });
      if (err != hipSuccess) break;
    }
    mtg_ctx::PipeSlot& s = ctx->pipe[c % S];
    const int64_t b0 = c * chunk, nb = std::min<int64_t>(chunk, batch - b0);
    char* dp = static_cast<char*>(s.dev);
    hipStream_t up = ctx->pipe_h2d;
    hipError_t e = hipMemcpyAsync(dp + o_vals, (const char*)values + b0 * s_vals, nb * s_vals,
                                  hipMemcpyHostToDevice, up);
    if (e == hipSuccess)
      e = hipMemcpyAsync(dp + o_mask, (const char*)mask + b0 * s_mask, nb * s_mask, hipMemcpyHostToDevice, up);
    if (e == hipSuccess)
      e = hipMemcpyAsync(dp + o_times, (const char*)times + b0 * s_times, nb * s_times, hipMemcpyHostToDevice, up);
    if (e == hipSuccess) e = hipEventRecord(s.in_done, up);
    if (e == hipSuccess) e = hipStreamWaitEvent(s.stream, s.in_done, 0);
    if (e == hipSuccess && free_out) e = hipMemsetAsync(dp + o_free, 0, nb * s_free, s.stream);
    if (e == hipSuccess) {
      mtg::SolveArgs a{};
      a.B = nb;
      a.K = K;
      a.D = D;
      a.r = r;
      a.n_cand = 1;
      a.values = reinterpret_cast<const double*>(dp + o_vals);
      a.mask = reinterpret_cast<const uint8_t*>(dp + o_mask);
      a.times = reinterpret_cast<const double*>(dp + o_times);
      a.coeffs = coeffs ? reinterpret_cast<double*>(dp + o_coef) : nullptr;
      a.free_out = free_out ? reinterpret_cast<double*>(dp + o_free) : nullptr;
      a.n_free_out = n_free_out ? reinterpret_cast<int32_t*>(dp + o_nfree) : nullptr;
      a.cost_out = cost_out ? reinterpret_cast<double*>(dp + o_cost) : nullptr;
      a.status = status ? reinterpret_cast<int32_t*>(dp + o_status) : nullptr;
      a.work = s_work ? reinterpret_cast<double*>(dp + o_work) : nullptr;
      a.work_bytes = (int64_t)s_work;
      e = mtg::launch_solve(N, a, s.stream, kflags);
    }
    if (e == hipSuccess) e = hipEventRecord(s.k_done, s.stream);
    if (e != hipSuccess) {
      fail(e, "pipelined H2D / launch");
      break;
    }
    std::lock_guard<std::mutex> g(m);
    launched = c + 1;
    cv.notify_all();
  }
  ctx->d2h_worker.wait();
  // nothing may still read or write the caller's arrays
  (void)hipStreamSynchronize(ctx->pipe_h2d);
  for (auto& s : ctx->pipe) (void)hipStreamSynchronize(s.stream);
  (void)hipStreamSynchronize(ctx->pipe_d2h);
  if (err != hipSuccess) return set_hip_error(ctx, err, err_what);
  // close the timed interval after the last D2H (every D2H is on pipe_d2h, in chunk order)
  MTG_HIP_TRY(ctx, hipEventRecord(ctx->pipe[(n_chunks - 1) % S].done, ctx->pipe_d2h));
  MTG_HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->pipe[(n_chunks - 1) % S].done, 0));
  MTG_HIP_TRY(ctx, time_end(ctx));
  MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MTG_OK;
}

// Shared body of solve / time-sweep: stage host buffers if needed, launch, copy back.
int run_solve(mtg_ctx* ctx, int N, int D, int K, int r, int64_t batch, const double* values,
              const uint8_t* mask, const double* times, double* coeffs, double* free_out,
              int32_t* n_free_out, double* cost_out, int32_t* status, int n_cand,
              const double* scales, unsigned flags) {
  const int V = K + 1, h = N / 2;
  const int64_t pairs = batch * n_cand;
  MTG_HIP_TRY(ctx, hipSetDevice(ctx->device));
  // (a time sweep passes scales, also with one candidate: it takes the single-stream path, which stages them)
  if (!(flags & (MTG_FLAG_DEVICE_PTRS | MTG_FLAG_SPLIT_KERNELS)) && n_cand == 1 && !scales &&
      (size_t)batch * (sizeof(double) * ((size_t)V * h * D + K + (size_t)K * D * N) + V) > kPipelineMinBytes) {
    // the chunks run the kernel the whole batch would (the default is the same at every batch size;
    // the explicit flag keeps it so)
    const unsigned kf = flags & (MTG_FLAG_GENERAL_KERNEL |
                                 MTG_FLAG_DL_KERNEL | MTG_FLAG_COLUMN_KERNEL);
    const int kk = mtg::solve_kernel(N, D, K, kf, r, batch);
    const unsigned pin = (kk == MTG_KERNEL_DL || kk == MTG_KERNEL_DLX) ? MTG_FLAG_DL_KERNEL : MTG_FLAG_COLUMN_KERNEL;
    const int rc = run_solve_pipelined(ctx, N, D, K, r, batch, values, mask, times, coeffs, free_out, n_free_out,
                                       cost_out, status, kf | pin);
    if (rc != kPipelineUnavailable) return rc;
  }
  mtg::SolveArgs a{};
  a.B = pairs;
  a.K = K;
  a.D = D;
  a.r = r;
  a.n_cand = n_cand;
  const bool dev = flags & MTG_FLAG_DEVICE_PTRS;
  const size_t b_vals = sizeof(double) * (size_t)batch * V * h * D;
  const size_t b_mask = sizeof(uint8_t) * (size_t)batch * V;
  const size_t b_times = sizeof(double) * (size_t)batch * K;
  const size_t b_scales = scales ? sizeof(double) * (size_t)n_cand : 0;
  const size_t b_coeffs = coeffs ? sizeof(double) * (size_t)pairs * K * D * N : 0;
  const size_t b_free = free_out ? sizeof(double) * (size_t)pairs * D * V * h : 0;
  const size_t b_nfree = n_free_out ? sizeof(int32_t) * (size_t)pairs : 0;
  const size_t b_cost = cost_out ? sizeof(double) * (size_t)pairs : 0;
  const size_t b_status = status ? sizeof(int32_t) * (size_t)pairs : 0;
  char* base = nullptr;
  size_t o_vals = 0, o_mask = 0, o_times = 0, o_scales = 0, o_coeffs = 0, o_free = 0, o_nfree = 0,
         o_cost = 0, o_status = 0, out_end = 0;
  bool pin = false;
  if (dev) {
    a.values = values;
    a.mask = mask;
    a.times = times;
    a.scales = scales;
    a.coeffs = coeffs;
    a.free_out = free_out;
    a.n_free_out = n_free_out;
    a.cost_out = cost_out;
    a.status = status;
  } else {
    size_t off = 0;
    o_vals = off; off = align_up(off + b_vals);
    o_mask = off; off = align_up(off + b_mask);
    o_times = off; off = align_up(off + b_times);
    o_scales = off; off = align_up(off + b_scales);
    o_coeffs = off; off = align_up(off + b_coeffs);
    o_free = off; off = align_up(off + b_free);
    o_nfree = off; off = align_up(off + b_nfree);
    o_cost = off; off = align_up(off + b_cost);
    o_status = off; off = align_up(off + b_status);
    MTG_HIP_TRY(ctx, ensure(&ctx->staging, &ctx->staging_bytes, std::max<size_t>(off, 256)));
    base = static_cast<char*>(ctx->staging);
    pin = off <= kPinnedMax;
    if (pin) {
      // small call (a drop-in PolynomialOptimization::solveLinear): pack the inputs into a pinned
      // mirror of the staging layout and move them with ONE DMA each way, instead of one pageable
      // copy per array (each of which the runtime bounces through its own pinned buffer)
      if (ctx->pinned_bytes < off) {
        if (ctx->pinned) MTG_HIP_TRY(ctx, hipHostFree(ctx->pinned));
        ctx->pinned = nullptr;
        ctx->pinned_bytes = 0;
        MTG_HIP_TRY(ctx, hipHostMalloc(&ctx->pinned, kPinnedMax, hipHostMallocDefault));
        ctx->pinned_bytes = kPinnedMax;
      }
      char* hp = static_cast<char*>(ctx->pinned);
      std::memcpy(hp + o_vals, values, b_vals);
      std::memcpy(hp + o_mask, mask, b_mask);
      std::memcpy(hp + o_times, times, b_times);
      if (scales) std::memcpy(hp + o_scales, scales, b_scales);
      MTG_HIP_TRY(ctx, hipMemcpyAsync(base, hp, o_coeffs, hipMemcpyHostToDevice, ctx->stream));
    } else {
      MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_vals, values, b_vals, hipMemcpyHostToDevice, ctx->stream));
      MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_mask, mask, b_mask, hipMemcpyHostToDevice, ctx->stream));
      MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_times, times, b_times, hipMemcpyHostToDevice, ctx->stream));
      if (scales)
        MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_scales, scales, b_scales, hipMemcpyHostToDevice, ctx->stream));
    }
    out_end = off;
    a.values = reinterpret_cast<const double*>(base + o_vals);
    a.mask = reinterpret_cast<const uint8_t*>(base + o_mask);
    a.times = reinterpret_cast<const double*>(base + o_times);
    a.scales = scales ? reinterpret_cast<const double*>(base + o_scales) : nullptr;
    a.coeffs = coeffs ? reinterpret_cast<double*>(base + o_coeffs) : nullptr;
    a.free_out = free_out ? reinterpret_cast<double*>(base + o_free) : nullptr;
    a.n_free_out = n_free_out ? reinterpret_cast<int32_t*>(base + o_nfree) : nullptr;
    a.cost_out = cost_out ? reinterpret_cast<double*>(base + o_cost) : nullptr;
    a.status = status ? reinterpret_cast<int32_t*>(base + o_status) : nullptr;
  }
  // From here on a failure must not return while a DMA may still read ctx->pinned (the next call
  // would overwrite it): the pinned path drains the stream before reporting any error.
  struct PinnedDrain {
    mtg_ctx* ctx;
    bool armed;
    ~PinnedDrain() {
      if (armed) (void)hipStreamSynchronize(ctx->stream);
    }
  } drain{ctx, pin};
  if (free_out && b_free) {
    // entries beyond n_free are left zero
    MTG_HIP_TRY(ctx, hipMemsetAsync(const_cast<double*>(a.free_out), 0, b_free, ctx->stream));
  }
  const unsigned ksel = flags & (MTG_FLAG_GENERAL_KERNEL | MTG_FLAG_DL_KERNEL | MTG_FLAG_COLUMN_KERNEL);
  const bool dlx = !(flags & MTG_FLAG_SPLIT_KERNELS) && mtg::solve_kernel(N, D, K, ksel, r, pairs) == MTG_KERNEL_DLX;
  if (dlx) {  // the long-chain DL kernel's workspace (and two launches: the timed region spans both)
    const size_t wb = mtg::dlx_workspace_bytes(N, D, K, pairs);
    MTG_HIP_TRY(ctx, ensure(&ctx->workspace, &ctx->workspace_bytes, std::max<size_t>(wb, 256)));
    a.work = static_cast<double*>(ctx->workspace);
    a.work_bytes = (int64_t)ctx->workspace_bytes;
  }
  MTG_HIP_TRY(ctx, time_begin(ctx, !(flags & MTG_FLAG_SPLIT_KERNELS) && !dlx));
  if (flags & MTG_FLAG_SPLIT_KERNELS) {
    const size_t ws = mtg::split_workspace_bytes(N, D, K, pairs);
    MTG_HIP_TRY(ctx, ensure(&ctx->workspace, &ctx->workspace_bytes, std::max<size_t>(ws, 256)));
    MTG_HIP_TRY(ctx, mtg::launch_solve_split(N, a, ctx->workspace, ctx->stream));
  } else {
    MTG_HIP_TRY(ctx, mtg::launch_solve(N, a, ctx->stream, ksel));
  }
  MTG_HIP_TRY(ctx, time_end(ctx));
  if (pin) {
    char* hp = static_cast<char*>(ctx->pinned);
    MTG_HIP_TRY(ctx, hipMemcpyAsync(hp + o_coeffs, base + o_coeffs, out_end - o_coeffs, hipMemcpyDeviceToHost,
                                    ctx->stream));
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (coeffs) std::memcpy(coeffs, hp + o_coeffs, b_coeffs);
    if (free_out) std::memcpy(free_out, hp + o_free, b_free);
    if (n_free_out) std::memcpy(n_free_out, hp + o_nfree, b_nfree);
    if (cost_out) std::memcpy(cost_out, hp + o_cost, b_cost);
    if (status) std::memcpy(status, hp + o_status, b_status);
    drain.armed = false;
  } else if (!dev) {
    if (coeffs) MTG_HIP_TRY(ctx, hipMemcpyAsync(coeffs, base + o_coeffs, b_coeffs, hipMemcpyDeviceToHost, ctx->stream));
    if (free_out) MTG_HIP_TRY(ctx, hipMemcpyAsync(free_out, base + o_free, b_free, hipMemcpyDeviceToHost, ctx->stream));
    if (n_free_out) MTG_HIP_TRY(ctx, hipMemcpyAsync(n_free_out, base + o_nfree, b_nfree, hipMemcpyDeviceToHost, ctx->stream));
    if (cost_out) MTG_HIP_TRY(ctx, hipMemcpyAsync(cost_out, base + o_cost, b_cost, hipMemcpyDeviceToHost, ctx->stream));
    if (status) MTG_HIP_TRY(ctx, hipMemcpyAsync(status, base + o_status, b_status, hipMemcpyDeviceToHost, ctx->stream));
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  } else if (!(flags & MTG_FLAG_ASYNC)) {
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  }
  return MTG_OK;
}

}  // namespace

extern "C" {

int mtg_abi_version(void) { return MTG_ABI_VERSION; }

int mtg_solve_kernel(int N, int D, int K, int derivative_to_optimize, unsigned flags) {
  if (N < 2 || N > 12 || (N % 2)) return MTG_ERR_UNSUPPORTED_N;
  if (derivative_to_optimize < 0 || derivative_to_optimize > N / 2 - 1) return MTG_ERR_BAD_DERIVATIVE;
  if (K < 1 || D < 1) return MTG_ERR_SIZE_MISMATCH;
  int lg, tpb;
  size_t lds;
  if (!mtg::solve_geometry(N, D, K, &lg, &lds, &tpb)) return MTG_ERR_TOO_LARGE;
  if (flags & MTG_FLAG_SPLIT_KERNELS) return MTG_KERNEL_SPLIT;
  return mtg::solve_kernel(N, D, K, flags, derivative_to_optimize);
}

int mtg_solve_kernel_batch(int N, int D, int K, int derivative_to_optimize, int64_t B, unsigned flags) {
  const int k = mtg_solve_kernel(N, D, K, derivative_to_optimize, flags);
  if (k < 0 || k == MTG_KERNEL_SPLIT || B < 0) return k;
  return mtg::solve_kernel(N, D, K, flags, derivative_to_optimize, B);
}

const char* mtg_status_string(int code) {
  switch (code) {
    case MTG_OK: return "ok";
    case MTG_ERR_INVALID_ARGUMENT: return "invalid argument";
    case MTG_ERR_UNSUPPORTED_N: return "unsupported N (even, 2..12)";
    case MTG_ERR_BAD_DERIVATIVE: return "derivative_to_optimize out of [0, N/2-1]";
    case MTG_ERR_SIZE_MISMATCH: return "size mismatch";
    case MTG_ERR_HIP: return "HIP runtime error";
    case MTG_ERR_NO_DEVICE: return "no HIP device";
    case MTG_ERR_OUT_OF_MEMORY: return "out of device memory";
    case MTG_ERR_TOO_LARGE: return "problem too large for the LDS-resident solver";
    default: return "unknown status";
  }
}

const char* mtg_last_error(mtg_ctx* ctx) { return ctx ? ctx->last_error.c_str() : "null context"; }

int mtg_device_count(int* count) {
  if (!count) return MTG_ERR_INVALID_ARGUMENT;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return e == hipErrorNoDevice ? MTG_ERR_NO_DEVICE : MTG_ERR_HIP;
  }
  *count = n;
  return MTG_OK;
}

int mtg_create(int device, mtg_ctx** out_ctx) {
  if (!out_ctx) return MTG_ERR_INVALID_ARGUMENT;
  *out_ctx = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return MTG_ERR_NO_DEVICE;
  if (device < 0 || device >= n) return MTG_ERR_INVALID_ARGUMENT;
  mtg_ctx* ctx = new (std::nothrow) mtg_ctx();
  if (!ctx) return MTG_ERR_OUT_OF_MEMORY;
  ctx->device = device;
  hipError_t e = hipSetDevice(device);
  // (MTG_HOST_WAIT=block: every wait of the process's HIP runtime on this device sleeps, including
  // the runtime's own waits inside pageable copies; measurement only, see host_wait_blocking)
  if (e == hipSuccess && host_wait_blocking()) (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = create_events(ctx, 1);
  if (e != hipSuccess) {
    mtg_destroy(ctx);
    return MTG_ERR_HIP;
  }
  ctx->stream = ctx->own_stream;
  *out_ctx = ctx;
  return MTG_OK;
}

int mtg_destroy(mtg_ctx* ctx) {
  if (!ctx) return MTG_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->staging) (void)hipFree(ctx->staging);
  if (ctx->workspace) (void)hipFree(ctx->workspace);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  destroy_pipe(ctx);
  destroy_events(ctx);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
  return MTG_OK;
}

int mtg_set_stream(mtg_ctx* ctx, void* hip_stream) {
  if (!ctx) return MTG_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->stream = static_cast<hipStream_t>(hip_stream);  // NULL = the HIP null stream
  return MTG_OK;
}

int mtg_reset_stream(mtg_ctx* ctx) {
  if (!ctx) return MTG_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->stream = ctx->own_stream;
  return MTG_OK;
}

void* mtg_get_stream(mtg_ctx* ctx) { return ctx ? static_cast<void*>(ctx->stream) : nullptr; }

int mtg_synchronize(mtg_ctx* ctx) {
  if (!ctx) return MTG_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(ctx->mu);
  MTG_HIP_TRY(ctx, hipSetDevice(ctx->device));
  MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MTG_OK;
}

int mtg_solve_linear_batch(mtg_ctx* ctx, int N, int D, int K, int derivative_to_optimize,
                           int64_t batch, const double* values, const uint8_t* fixed_mask,
                           const double* times, double* coeffs, double* free_out,
                           int32_t* n_free_out, double* cost_out, int32_t* status,
                           unsigned flags) {
  int rc = check_shape(ctx, N, D, K, derivative_to_optimize, batch);
  if (rc != MTG_OK) return rc;
  if (batch == 0) return MTG_OK;
  if (!values || !fixed_mask || !times)
    return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "values, fixed_mask and times are required");
  std::lock_guard<std::mutex> g(ctx->mu);
  if (ctx->inject_rc) {  // (diagnostics: mtg_debug_fail_next_solve)
    const int code = ctx->inject_rc;
    ctx->inject_rc = 0;
    return set_error(ctx, code, "injected fault (mtg_debug_fail_next_solve)");
  }
  return run_solve(ctx, N, D, K, derivative_to_optimize, batch, values, fixed_mask, times, coeffs,
                   free_out, n_free_out, cost_out, status, 1, nullptr, flags);
}

int mtg_debug_fail_next_solve(mtg_ctx* ctx, int code) {
  if (!ctx || code >= 0) return MTG_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->inject_rc = code;
  return MTG_OK;
}

int mtg_shard_range(int64_t batch, int n_shards, int shard, int64_t* begin, int64_t* end) {
  if (batch < 0 || n_shards < 1 || shard < 0 || shard >= n_shards || !begin || !end) return MTG_ERR_INVALID_ARGUMENT;
  const int64_t per = (batch + n_shards - 1) / n_shards;  // ceil(B / G), SURVEY.md 8(e)
  *begin = std::min<int64_t>(batch, (int64_t)shard * per);
  *end = std::min<int64_t>(batch, *begin + per);
  return MTG_OK;
}

int mtg_solve_linear_batch_multi(mtg_ctx* const* ctxs, int n_ctxs, int N, int D, int K, int derivative_to_optimize,
                                 int64_t batch, const double* values, const uint8_t* fixed_mask,
                                 const double* times, double* coeffs, double* free_out, int32_t* n_free_out,
                                 double* cost_out, int32_t* status, unsigned flags) {
  if (!ctxs || n_ctxs < 1) return MTG_ERR_INVALID_ARGUMENT;
  for (int g = 0; g < n_ctxs; ++g)
    if (!ctxs[g]) return MTG_ERR_INVALID_ARGUMENT;
  mtg_ctx* c0 = ctxs[0];
  if (flags & (MTG_FLAG_DEVICE_PTRS | MTG_FLAG_ASYNC))
    return set_error(c0, MTG_ERR_INVALID_ARGUMENT, "multi-device solves take host arrays and are synchronous");
  int rc = check_shape(c0, N, D, K, derivative_to_optimize, batch);
  if (rc != MTG_OK) return rc;
  if (batch == 0) return MTG_OK;
  if (!values || !fixed_mask || !times)
    return set_error(c0, MTG_ERR_INVALID_ARGUMENT, "values, fixed_mask and times are required");
  const int V = K + 1, h = N / 2;
  const size_t s_vals = (size_t)V * h * D, s_coef = (size_t)K * D * N, s_free = (size_t)D * V * h;
  std::vector<int> rcs(n_ctxs, MTG_OK);
  // every shard runs the kernel the whole batch would on one device (the default no longer depends on
  // the batch size -- the DL kernel for N = 10 / K = 10 and N = 12 / K = 20 at every size -- but the
  // flag keeps the choice explicit), so the result does not depend on the number of devices
  if (!(flags & MTG_FLAG_SPLIT_KERNELS))
  {
    const int kk = mtg::solve_kernel(N, D, K, flags, derivative_to_optimize, batch);
    flags |= (kk == MTG_KERNEL_DL || kk == MTG_KERNEL_DLX) ? MTG_FLAG_DL_KERNEL : MTG_FLAG_COLUMN_KERNEL;
  }
  auto shard = [&](int g) {
    int64_t b0 = 0, b1 = 0;
    mtg_shard_range(batch, n_ctxs, g, &b0, &b1);
    if (b1 <= b0) return;
    rcs[g] = mtg_solve_linear_batch(ctxs[g], N, D, K, derivative_to_optimize, b1 - b0, values + b0 * s_vals,
                                    fixed_mask + b0 * V, times + b0 * K, coeffs ? coeffs + b0 * s_coef : nullptr,
                                    free_out ? free_out + b0 * s_free : nullptr, n_free_out ? n_free_out + b0 : nullptr,
                                    cost_out ? cost_out + b0 : nullptr, status ? status + b0 : nullptr, flags);
  };
  // one host thread per context: each drives its device's staging or chunk pipeline and writes its
  // disjoint slice of the outputs (no collective); shard 0 runs on this thread
  std::vector<std::thread> pool;
  for (int g = 1; g < n_ctxs; ++g) {
    try {
      pool.emplace_back(shard, g);
    } catch (...) {  // no thread: solve this shard here instead
      shard(g);
    }
  }
  shard(0);
  for (auto& t : pool) t.join();
  for (int g = 0; g < n_ctxs; ++g) {
    if (rcs[g] == MTG_OK) continue;
    std::string what;
    {
      std::lock_guard<std::mutex> l(ctxs[g]->mu);
      what = ctxs[g]->last_error;
    }
    std::lock_guard<std::mutex> l(c0->mu);
    c0->last_error = "shard " + std::to_string(g) + " of " + std::to_string(n_ctxs) + ": " + what;
    return rcs[g];
  }
  return MTG_OK;
}

int mtg_time_sweep_batch(mtg_ctx* ctx, int N, int D, int K, int derivative_to_optimize,
                         int64_t batch, const double* values, const uint8_t* fixed_mask,
                         const double* times, int n_candidates, const double* scales,
                         double* cost_out, int32_t* status, unsigned flags) {
  int rc = check_shape(ctx, N, D, K, derivative_to_optimize, batch);
  if (rc != MTG_OK) return rc;
  if (n_candidates < 1) return set_error(ctx, MTG_ERR_SIZE_MISMATCH, "n_candidates must be >= 1");
  if (batch == 0) return MTG_OK;
  if (!values || !fixed_mask || !times || !scales || !cost_out)
    return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "values, fixed_mask, times, scales, cost_out are required");
  std::lock_guard<std::mutex> g(ctx->mu);
  return run_solve(ctx, N, D, K, derivative_to_optimize, batch, values, fixed_mask, times, nullptr,
                   nullptr, nullptr, cost_out, status, n_candidates, scales,
                   flags);
}

int mtg_cost_at_times_batch(mtg_ctx* ctx, int N, int D, int K, int derivative_to_optimize,
                            int64_t batch, const double* vertex_values, const uint8_t* fixed_mask,
                            const double* times, int n_candidates, const double* scales,
                            double* cost_out, double* grad_out, unsigned flags) {
  int rc = check_shape(ctx, N, D, K, derivative_to_optimize, batch);
  if (rc != MTG_OK) return rc;
  if (n_candidates < 1) return set_error(ctx, MTG_ERR_SIZE_MISMATCH, "n_candidates must be >= 1");
  if (batch == 0) return MTG_OK;
  if (!vertex_values || !times || !scales || !cost_out || (grad_out && !fixed_mask))
    return set_error(ctx, MTG_ERR_INVALID_ARGUMENT,
                     "vertex_values, times, scales, cost_out are required; grad_out needs fixed_mask");
  if (mtg::cost_lds_bytes(N, D, K) > 64 * 1024)
    return set_error(ctx, MTG_ERR_TOO_LARGE, "per-trajectory cost tables exceed LDS (reduce K or D)");
  std::lock_guard<std::mutex> g(ctx->mu);
  MTG_HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int V = K + 1, h = N / 2, C = n_candidates;
  const size_t b_vals = sizeof(double) * (size_t)batch * V * h * D, b_mask = grad_out ? (size_t)batch * V : 0,
               b_times = sizeof(double) * (size_t)batch * K, b_scales = sizeof(double) * (size_t)C * K,
               b_cost = sizeof(double) * (size_t)batch * C,
               b_grad = grad_out ? sizeof(double) * (size_t)batch * C * D * V * h : 0;
  const double* d_vals = vertex_values;
  const uint8_t* d_mask = fixed_mask;
  const double *d_times = times, *d_scales = scales;
  double *d_cost = cost_out, *d_grad = grad_out;
  const bool dev = flags & MTG_FLAG_DEVICE_PTRS;
  char* base = nullptr;
  size_t o_cost = 0, o_grad = 0;
  if (!dev) {
    size_t off = 0;
    const size_t o_vals = off; off = align_up(off + b_vals);
    const size_t o_mask = off; off = align_up(off + b_mask);
    const size_t o_times = off; off = align_up(off + b_times);
    const size_t o_scales = off; off = align_up(off + b_scales);
    o_cost = off; off = align_up(off + b_cost);
    o_grad = off; off = align_up(off + b_grad);
    MTG_HIP_TRY(ctx, ensure(&ctx->staging, &ctx->staging_bytes, std::max<size_t>(off, 256)));
    base = static_cast<char*>(ctx->staging);
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_vals, vertex_values, b_vals, hipMemcpyHostToDevice, ctx->stream));
    if (b_mask) MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_mask, fixed_mask, b_mask, hipMemcpyHostToDevice, ctx->stream));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_times, times, b_times, hipMemcpyHostToDevice, ctx->stream));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_scales, scales, b_scales, hipMemcpyHostToDevice, ctx->stream));
    d_vals = reinterpret_cast<const double*>(base + o_vals);
    d_mask = b_mask ? reinterpret_cast<const uint8_t*>(base + o_mask) : nullptr;
    d_times = reinterpret_cast<const double*>(base + o_times);
    d_scales = reinterpret_cast<const double*>(base + o_scales);
    d_cost = reinterpret_cast<double*>(base + o_cost);
    d_grad = grad_out ? reinterpret_cast<double*>(base + o_grad) : nullptr;
  }
  if (d_grad) MTG_HIP_TRY(ctx, hipMemsetAsync(d_grad, 0, b_grad, ctx->stream));
  MTG_HIP_TRY(ctx, time_begin(ctx));
  MTG_HIP_TRY(ctx, mtg::launch_cost_at_times(N, derivative_to_optimize, d_vals, d_mask, d_times, d_scales, d_cost,
                                             d_grad, batch, K, D, C, ctx->stream));
  MTG_HIP_TRY(ctx, time_end(ctx));
  if (!dev) {
    MTG_HIP_TRY(ctx, hipMemcpyAsync(cost_out, base + o_cost, b_cost, hipMemcpyDeviceToHost, ctx->stream));
    if (grad_out) MTG_HIP_TRY(ctx, hipMemcpyAsync(grad_out, base + o_grad, b_grad, hipMemcpyDeviceToHost, ctx->stream));
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  } else if (!(flags & MTG_FLAG_ASYNC)) {
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  }
  return MTG_OK;
}

int mtg_time_jacobian_batch(mtg_ctx* ctx, int N, int D, int K, int derivative_to_optimize,
                            int64_t batch, const double* vertex_values, const double* times,
                            int n_candidates, const double* scales, double increment_time,
                            double* cost_out, double* jac_out, unsigned flags) {
  int rc = check_shape(ctx, N, D, K, derivative_to_optimize, batch);
  if (rc != MTG_OK) return rc;
  if (n_candidates < 1) return set_error(ctx, MTG_ERR_SIZE_MISMATCH, "n_candidates must be >= 1");
  if (!(increment_time >= 0.0) || increment_time > DBL_MAX)
    return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "increment_time must be finite and >= 0");
  if (batch == 0) return MTG_OK;
  if (!vertex_values || !times || !scales || !cost_out)
    return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "vertex_values, times, scales, cost_out are required");
  if (mtg::time_jacobian_lds_bytes(N, D, K, n_candidates) > 160 * 1024)
    return set_error(ctx, MTG_ERR_TOO_LARGE, "per-block cost tables exceed LDS (reduce K or D)");
  std::lock_guard<std::mutex> g(ctx->mu);
  MTG_HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int V = K + 1, h = N / 2, C = n_candidates;
  const size_t b_vals = sizeof(double) * (size_t)batch * V * h * D, b_times = sizeof(double) * (size_t)batch * K,
               b_scales = sizeof(double) * (size_t)C * K, b_cost = sizeof(double) * (size_t)batch * C,
               b_jac = jac_out ? sizeof(double) * (size_t)batch * C * K : 0;
  const double *d_vals = vertex_values, *d_times = times, *d_scales = scales;
  double *d_cost = cost_out, *d_jac = jac_out;
  const bool dev = flags & MTG_FLAG_DEVICE_PTRS;
  char* base = nullptr;
  size_t o_cost = 0, o_jac = 0;
  if (!dev) {
    size_t off = 0;
    const size_t o_vals = off; off = align_up(off + b_vals);
    const size_t o_times = off; off = align_up(off + b_times);
    const size_t o_scales = off; off = align_up(off + b_scales);
    o_cost = off; off = align_up(off + b_cost);
    o_jac = off; off = align_up(off + b_jac);
    MTG_HIP_TRY(ctx, ensure(&ctx->staging, &ctx->staging_bytes, std::max<size_t>(off, 256)));
    base = static_cast<char*>(ctx->staging);
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_vals, vertex_values, b_vals, hipMemcpyHostToDevice, ctx->stream));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_times, times, b_times, hipMemcpyHostToDevice, ctx->stream));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_scales, scales, b_scales, hipMemcpyHostToDevice, ctx->stream));
    d_vals = reinterpret_cast<const double*>(base + o_vals);
    d_times = reinterpret_cast<const double*>(base + o_times);
    d_scales = reinterpret_cast<const double*>(base + o_scales);
    d_cost = reinterpret_cast<double*>(base + o_cost);
    d_jac = jac_out ? reinterpret_cast<double*>(base + o_jac) : nullptr;
  }
  MTG_HIP_TRY(ctx, time_begin(ctx));
  MTG_HIP_TRY(ctx, mtg::launch_time_jacobian(N, derivative_to_optimize, d_vals, d_times, d_scales, d_cost, d_jac,
                                             increment_time, batch, K, D, C, ctx->stream));
  MTG_HIP_TRY(ctx, time_end(ctx));
  if (!dev) {
    MTG_HIP_TRY(ctx, hipMemcpyAsync(cost_out, base + o_cost, b_cost, hipMemcpyDeviceToHost, ctx->stream));
    if (jac_out) MTG_HIP_TRY(ctx, hipMemcpyAsync(jac_out, base + o_jac, b_jac, hipMemcpyDeviceToHost, ctx->stream));
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  } else if (!(flags & MTG_FLAG_ASYNC)) {
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  }
  return MTG_OK;
}

namespace {

// Shared body of the two vertex <-> coefficient maps: [B][V][h][D] <-> [B][K][D][N].
int run_vertex_map(mtg_ctx* ctx, bool to_coeffs, int N, int D, int K, int64_t batch, const double* in,
                   const double* times, double* out, unsigned flags) {
  if (!ctx) return MTG_ERR_INVALID_ARGUMENT;
  if (N < 2 || N > 12 || (N % 2)) return set_error(ctx, MTG_ERR_UNSUPPORTED_N, "N must be even and in [2, 12]");
  if (K < 1 || D < 1 || batch < 0) return set_error(ctx, MTG_ERR_SIZE_MISMATCH, "need K >= 1, D >= 1, batch >= 0");
  if (!mtg::vertex_map_fits(N, D, K))
    return set_error(ctx, MTG_ERR_TOO_LARGE, "per-trajectory arrays exceed the LDS staging (reduce K or D)");
  if (batch == 0) return MTG_OK;
  if (!in || !times || !out) return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "input, times and output are required");
  std::lock_guard<std::mutex> g(ctx->mu);
  MTG_HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int V = K + 1, h = N / 2;
  const size_t b_vals = sizeof(double) * (size_t)batch * V * h * D, b_coef = sizeof(double) * (size_t)batch * K * D * N,
               b_times = sizeof(double) * (size_t)batch * K;
  const size_t b_in = to_coeffs ? b_vals : b_coef, b_out = to_coeffs ? b_coef : b_vals;
  const double *d_in = in, *d_times = times;
  double* d_out = out;
  const bool dev = flags & MTG_FLAG_DEVICE_PTRS;
  char* base = nullptr;
  size_t o_out = 0;
  if (!dev) {
    size_t off = 0;
    const size_t o_in = off; off = align_up(off + b_in);
    const size_t o_times = off; off = align_up(off + b_times);
    o_out = off; off = align_up(off + b_out);
    MTG_HIP_TRY(ctx, ensure(&ctx->staging, &ctx->staging_bytes, std::max<size_t>(off, 256)));
    base = static_cast<char*>(ctx->staging);
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_in, in, b_in, hipMemcpyHostToDevice, ctx->stream));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_times, times, b_times, hipMemcpyHostToDevice, ctx->stream));
    d_in = reinterpret_cast<const double*>(base + o_in);
    d_times = reinterpret_cast<const double*>(base + o_times);
    d_out = reinterpret_cast<double*>(base + o_out);
  }
  MTG_HIP_TRY(ctx, time_begin(ctx));
  MTG_HIP_TRY(ctx, mtg::launch_vertex_map(to_coeffs, N, d_in, d_times, d_out, batch, K, D, ctx->stream));
  MTG_HIP_TRY(ctx, time_end(ctx));
  if (!dev) {
    MTG_HIP_TRY(ctx, hipMemcpyAsync(out, base + o_out, b_out, hipMemcpyDeviceToHost, ctx->stream));
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  } else if (!(flags & MTG_FLAG_ASYNC)) {
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  }
  return MTG_OK;
}

}  // namespace

int mtg_coefficients_from_vertices_batch(mtg_ctx* ctx, int N, int D, int K, int64_t batch,
                                         const double* vertex_values, const double* times, double* coeffs,
                                         unsigned flags) {
  return run_vertex_map(ctx, true, N, D, K, batch, vertex_values, times, coeffs, flags);
}

int mtg_vertex_derivatives_batch(mtg_ctx* ctx, int N, int D, int K, int64_t batch, const double* coeffs,
                                 const double* times, double* vertex_values, unsigned flags) {
  return run_vertex_map(ctx, false, N, D, K, batch, coeffs, times, vertex_values, flags);
}

int mtg_min_max_magnitude_batch(mtg_ctx* ctx, int N, int D, int K, int64_t batch, const double* coeffs,
                                const double* times, int derivative, uint32_t dimension_mask,
                                mtg_extremum* minimum, mtg_extremum* maximum, unsigned flags) {
  if (!ctx) return MTG_ERR_INVALID_ARGUMENT;
  if (N < 2 || N > 12 || (N % 2)) return set_error(ctx, MTG_ERR_UNSUPPORTED_N, "N must be even and in [2, 12]");
  if (K < 1 || D < 1 || batch < 0) return set_error(ctx, MTG_ERR_SIZE_MISMATCH, "need K >= 1, D >= 1, batch >= 0");
  if (K > 256) return set_error(ctx, MTG_ERR_TOO_LARGE, "K must be <= 256");
  if (derivative < 0 || derivative > N - 2)
    return set_error(ctx, MTG_ERR_BAD_DERIVATIVE, "derivative must be in [0, N-2] (polynomial.cpp:62-65)");
  const uint32_t all = D >= 32 ? 0xffffffffu : ((1u << D) - 1u);
  const uint32_t dims = dimension_mask ? dimension_mask : all;
  if (D > 32 || (dims & ~all)) return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "dimension_mask out of range");
  if (batch == 0) return MTG_OK;
  if (!coeffs || !times) return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "coeffs and times are required");
  std::lock_guard<std::mutex> g(ctx->mu);
  MTG_HIP_TRY(ctx, hipSetDevice(ctx->device));
  const size_t b_coef = sizeof(double) * (size_t)batch * K * D * N, b_times = sizeof(double) * (size_t)batch * K,
               b_ext = sizeof(mtg_extremum) * (size_t)batch;
  const double *d_coef = coeffs, *d_times = times;
  mtg_extremum *d_min = minimum, *d_max = maximum;
  const bool dev = flags & MTG_FLAG_DEVICE_PTRS;
  char* base = nullptr;
  size_t o_min = 0, o_max = 0;
  if (!dev) {
    size_t off = 0;
    const size_t o_coef = off; off = align_up(off + b_coef);
    const size_t o_times = off; off = align_up(off + b_times);
    o_min = off; off = align_up(off + b_ext);
    o_max = off; off = align_up(off + b_ext);
    MTG_HIP_TRY(ctx, ensure(&ctx->staging, &ctx->staging_bytes, std::max<size_t>(off, 256)));
    base = static_cast<char*>(ctx->staging);
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_coef, coeffs, b_coef, hipMemcpyHostToDevice, ctx->stream));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_times, times, b_times, hipMemcpyHostToDevice, ctx->stream));
    d_coef = reinterpret_cast<const double*>(base + o_coef);
    d_times = reinterpret_cast<const double*>(base + o_times);
    d_min = minimum ? reinterpret_cast<mtg_extremum*>(base + o_min) : nullptr;
    d_max = maximum ? reinterpret_cast<mtg_extremum*>(base + o_max) : nullptr;
  }
  MTG_HIP_TRY(ctx, time_begin(ctx));
  MTG_HIP_TRY(ctx, mtg::launch_min_max_magnitude(N, d_coef, d_times, batch, K, D, derivative, dims, d_min, d_max,
                                                 ctx->stream));
  MTG_HIP_TRY(ctx, time_end(ctx));
  if (!dev) {
    if (minimum) MTG_HIP_TRY(ctx, hipMemcpyAsync(minimum, base + o_min, b_ext, hipMemcpyDeviceToHost, ctx->stream));
    if (maximum) MTG_HIP_TRY(ctx, hipMemcpyAsync(maximum, base + o_max, b_ext, hipMemcpyDeviceToHost, ctx->stream));
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  } else if (!(flags & MTG_FLAG_ASYNC)) {
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  }
  return MTG_OK;
}

int mtg_evaluate_range_batch(mtg_ctx* ctx, int N, int D, int K, int64_t batch,
                             const double* coeffs, const double* times, double t_start,
                             double t_end, double dt, int derivative, int64_t* counts,
                             const int64_t* offsets, double* out, double* sample_times,
                             unsigned flags) {
  if (!ctx) return MTG_ERR_INVALID_ARGUMENT;
  if (N < 2 || N > 12 || (N % 2)) return set_error(ctx, MTG_ERR_UNSUPPORTED_N, "N must be even and in [2, 12]");
  if (K < 1 || D < 1 || batch < 0) return set_error(ctx, MTG_ERR_SIZE_MISMATCH, "need K >= 1, D >= 1, batch >= 0");
  if (!(dt > 0.0) || derivative < 0)
    return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "dt must be > 0 and derivative >= 0");
  if (batch == 0) return MTG_OK;
  if (!times || !counts || (out && (!coeffs || !offsets)))
    return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "times and counts required; out needs coeffs and offsets");
  std::lock_guard<std::mutex> g(ctx->mu);
  MTG_HIP_TRY(ctx, hipSetDevice(ctx->device));
  const bool dev = flags & MTG_FLAG_DEVICE_PTRS;
  if (dev) {
    if (!out) {
      MTG_HIP_TRY(ctx, mtg::launch_eval_count(N, D, K, batch, times, t_start, t_end, dt, counts, ctx->stream));
    } else {
      int cap = 0;
      const size_t wsb = mtg::eval_workspace_bytes(K, batch, &cap);
      MTG_HIP_TRY(ctx, ensure(&ctx->workspace, &ctx->workspace_bytes, std::max<size_t>(wsb, 256)));
      MTG_HIP_TRY(ctx, time_begin(ctx, false));  // two kernels: the run table, then the samples
      MTG_HIP_TRY(ctx, mtg::launch_eval_range(N, D, K, batch, coeffs, times, t_start, t_end, dt, derivative,
                                              counts, offsets, out, sample_times, ctx->workspace, cap,
                                              ctx->stream));
      MTG_HIP_TRY(ctx, time_end(ctx));
    }
    if (!(flags & MTG_FLAG_ASYNC)) MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return MTG_OK;
  }
  // Host pointers: stage everything.
  const size_t b_times = sizeof(double) * (size_t)batch * K;
  const size_t b_coeffs = coeffs ? sizeof(double) * (size_t)batch * K * D * N : 0;
  const size_t b_counts = sizeof(int64_t) * (size_t)batch;
  int64_t total = 0;
  if (out) {
    for (int64_t b = 0; b < batch; ++b) total = std::max<int64_t>(total, offsets[b] + counts[b]);
  }
  const size_t b_out = out ? sizeof(double) * (size_t)total * D : 0;
  const size_t b_st = (out && sample_times) ? sizeof(double) * (size_t)total : 0;
  size_t off = 0;
  const size_t o_times = off; off = align_up(off + b_times);
  const size_t o_coeffs = off; off = align_up(off + b_coeffs);
  const size_t o_counts = off; off = align_up(off + b_counts);
  const size_t o_offsets = off; off = align_up(off + b_counts);
  const size_t o_out = off; off = align_up(off + b_out);
  const size_t o_st = off; off = align_up(off + b_st);
  MTG_HIP_TRY(ctx, ensure(&ctx->staging, &ctx->staging_bytes, std::max<size_t>(off, 256)));
  char* base = static_cast<char*>(ctx->staging);
  MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_times, times, b_times, hipMemcpyHostToDevice, ctx->stream));
  if (!out) {
    MTG_HIP_TRY(ctx, mtg::launch_eval_count(N, D, K, batch, reinterpret_cast<double*>(base + o_times), t_start,
                                            t_end, dt, reinterpret_cast<int64_t*>(base + o_counts), ctx->stream));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(counts, base + o_counts, b_counts, hipMemcpyDeviceToHost, ctx->stream));
  } else {
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_coeffs, coeffs, b_coeffs, hipMemcpyHostToDevice, ctx->stream));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_offsets, offsets, b_counts, hipMemcpyHostToDevice, ctx->stream));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_counts, counts, b_counts, hipMemcpyHostToDevice, ctx->stream));
    int cap = 0;
    const size_t wsb = mtg::eval_workspace_bytes(K, batch, &cap);
    MTG_HIP_TRY(ctx, ensure(&ctx->workspace, &ctx->workspace_bytes, std::max<size_t>(wsb, 256)));
    MTG_HIP_TRY(ctx, time_begin(ctx, false));
    MTG_HIP_TRY(ctx, mtg::launch_eval_range(N, D, K, batch, reinterpret_cast<double*>(base + o_coeffs),
                                            reinterpret_cast<double*>(base + o_times), t_start, t_end, dt,
                                            derivative, reinterpret_cast<int64_t*>(base + o_counts),
                                            reinterpret_cast<int64_t*>(base + o_offsets),
                                            reinterpret_cast<double*>(base + o_out),
                                            sample_times ? reinterpret_cast<double*>(base + o_st) : nullptr,
                                            ctx->workspace, cap, ctx->stream));
    MTG_HIP_TRY(ctx, time_end(ctx));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(out, base + o_out, b_out, hipMemcpyDeviceToHost, ctx->stream));
    if (sample_times) MTG_HIP_TRY(ctx, hipMemcpyAsync(sample_times, base + o_st, b_st, hipMemcpyDeviceToHost, ctx->stream));
  }
  MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MTG_OK;
}

int mtg_evaluate_range_batch_full(mtg_ctx* ctx, int N, int D, int K, int64_t batch, const double* coeffs,
                                  const double* times, double t_start, double t_end, double dt, int derivative,
                                  int64_t* counts, int64_t* offsets, int64_t* total, double* out,
                                  double* sample_times, int64_t capacity, unsigned flags) {
  if (!ctx) return MTG_ERR_INVALID_ARGUMENT;
  if (N < 2 || N > 12 || (N % 2)) return set_error(ctx, MTG_ERR_UNSUPPORTED_N, "N must be even and in [2, 12]");
  if (K < 1 || D < 1 || batch < 0 || capacity < 0)
    return set_error(ctx, MTG_ERR_SIZE_MISMATCH, "need K >= 1, D >= 1, batch >= 0, capacity >= 0");
  if (!(dt > 0.0) || derivative < 0)
    return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "dt must be > 0 and derivative >= 0");
  if (!coeffs || !times || !counts || !offsets || !total || (capacity > 0 && !out))
    return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "coeffs, times, counts, offsets, total and out are required");
  std::lock_guard<std::mutex> g(ctx->mu);
  MTG_HIP_TRY(ctx, hipSetDevice(ctx->device));
  const bool dev = flags & MTG_FLAG_DEVICE_PTRS;
  if (batch == 0) {
    if (dev) MTG_HIP_TRY(ctx, hipMemsetAsync(total, 0, sizeof(int64_t), ctx->stream));
    else *total = 0;
    return MTG_OK;
  }
  int cap = 0;
  const size_t wsb = mtg::eval_full_workspace_bytes(K, batch, &cap);
  MTG_HIP_TRY(ctx, ensure(&ctx->workspace, &ctx->workspace_bytes, std::max<size_t>(wsb, 256)));
  int64_t* d_total_ws = reinterpret_cast<int64_t*>(static_cast<char*>(ctx->workspace) + wsb - sizeof(int64_t));
  if (dev) {
    // counts, offsets (in-block prefix, then final) and the total, then the samples: four kernels on
    // the stream, no host round trip in between
    MTG_HIP_TRY(ctx, time_begin(ctx, false));
    MTG_HIP_TRY(ctx, mtg::launch_eval_runs_counts(K, batch, times, t_start, t_end, dt, counts, offsets,
                                                  ctx->workspace, cap, total, ctx->stream));
    MTG_HIP_TRY(ctx, mtg::launch_eval_range(N, D, K, batch, coeffs, times, t_start, t_end, dt, derivative, counts,
                                            offsets, out, sample_times, ctx->workspace, cap, ctx->stream, true,
                                            offsets, capacity, total));
    MTG_HIP_TRY(ctx, time_end(ctx));
    if (flags & MTG_FLAG_ASYNC) return MTG_OK;
    int64_t tot = 0;
    MTG_HIP_TRY(ctx, hipMemcpyAsync(&tot, total, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (tot > capacity) {
      char buf[160];
      snprintf(buf, sizeof(buf), "evaluateRange needs %lld samples, capacity is %lld",
               (long long)tot, (long long)capacity);
      return set_error(ctx, MTG_ERR_TOO_LARGE, buf);
    }
    return MTG_OK;
  }
  // host arrays: counts and offsets first (one 8-B read of the total sizes the staging), then the
  // samples straight into staging sized to the total
  const size_t b_coef = sizeof(double) * (size_t)batch * K * D * N, b_times = sizeof(double) * (size_t)batch * K,
               b_cnt = sizeof(int64_t) * (size_t)batch;
  size_t off = 0;
  const size_t o_times = off; off = align_up(off + b_times);
  const size_t o_coef = off; off = align_up(off + b_coef);
  const size_t o_cnt = off; off = align_up(off + b_cnt);
  const size_t o_offs = off; off = align_up(off + b_cnt);
  const size_t in_end = off;
  MTG_HIP_TRY(ctx, ensure(&ctx->staging, &ctx->staging_bytes, std::max<size_t>(in_end, 256)));
  char* base = static_cast<char*>(ctx->staging);
  MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_times, times, b_times, hipMemcpyHostToDevice, ctx->stream));
  MTG_HIP_TRY(ctx, hipMemcpyAsync(base + o_coef, coeffs, b_coef, hipMemcpyHostToDevice, ctx->stream));
  int64_t* d_cnt = reinterpret_cast<int64_t*>(base + o_cnt);
  int64_t* d_offs = reinterpret_cast<int64_t*>(base + o_offs);
  MTG_HIP_TRY(ctx, time_begin(ctx, false));
  MTG_HIP_TRY(ctx, mtg::launch_eval_runs_counts(K, batch, reinterpret_cast<const double*>(base + o_times), t_start,
                                                t_end, dt, d_cnt, d_offs, ctx->workspace, cap, d_total_ws,
                                                ctx->stream));
  int64_t tot = 0;
  MTG_HIP_TRY(ctx, hipMemcpyAsync(&tot, d_total_ws, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  *total = tot;
  const size_t b_out = sizeof(double) * (size_t)(tot <= capacity ? tot : 0) * D;
  const size_t b_st = sample_times ? sizeof(double) * (size_t)(tot <= capacity ? tot : 0) : 0;
  const size_t o_out = in_end, o_st = align_up(o_out + b_out), all_end = align_up(o_st + b_st);
  if (all_end > ctx->staging_bytes) {  // grow, keeping the staged inputs and counts
    void* grown = nullptr;
    MTG_HIP_TRY(ctx, hipMalloc(&grown, all_end));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(grown, ctx->staging, in_end, hipMemcpyDeviceToDevice, ctx->stream));
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    MTG_HIP_TRY(ctx, hipFree(ctx->staging));
    ctx->staging = grown;
    ctx->staging_bytes = all_end;
    base = static_cast<char*>(grown);
    d_cnt = reinterpret_cast<int64_t*>(base + o_cnt);
    d_offs = reinterpret_cast<int64_t*>(base + o_offs);
  }
  if (tot > capacity) {  // counts, final offsets and the total for the caller's retry; no samples
    MTG_HIP_TRY(ctx, mtg::launch_eval_range(N, D, K, batch, reinterpret_cast<const double*>(base + o_coef),
                                            reinterpret_cast<const double*>(base + o_times), t_start, t_end, dt,
                                            derivative, d_cnt, d_offs, nullptr, nullptr, ctx->workspace, cap,
                                            ctx->stream, true, d_offs, 0));
    MTG_HIP_TRY(ctx, time_end(ctx));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(counts, d_cnt, b_cnt, hipMemcpyDeviceToHost, ctx->stream));
    MTG_HIP_TRY(ctx, hipMemcpyAsync(offsets, d_offs, b_cnt, hipMemcpyDeviceToHost, ctx->stream));
    MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    char buf[160];
    snprintf(buf, sizeof(buf), "evaluateRange needs %lld samples, capacity is %lld", (long long)tot,
             (long long)capacity);
    return set_error(ctx, MTG_ERR_TOO_LARGE, buf);
  }
  MTG_HIP_TRY(ctx, mtg::launch_eval_range(N, D, K, batch, reinterpret_cast<const double*>(base + o_coef),
                                          reinterpret_cast<const double*>(base + o_times), t_start, t_end, dt,
                                          derivative, d_cnt, d_offs, reinterpret_cast<double*>(base + o_out),
                                          sample_times ? reinterpret_cast<double*>(base + o_st) : nullptr,
                                          ctx->workspace, cap, ctx->stream, true, d_offs, capacity));
  MTG_HIP_TRY(ctx, time_end(ctx));
  MTG_HIP_TRY(ctx, hipMemcpyAsync(counts, d_cnt, b_cnt, hipMemcpyDeviceToHost, ctx->stream));
  MTG_HIP_TRY(ctx, hipMemcpyAsync(offsets, d_offs, b_cnt, hipMemcpyDeviceToHost, ctx->stream));
  if (b_out) MTG_HIP_TRY(ctx, hipMemcpyAsync(out, base + o_out, b_out, hipMemcpyDeviceToHost, ctx->stream));
  if (b_st) MTG_HIP_TRY(ctx, hipMemcpyAsync(sample_times, base + o_st, b_st, hipMemcpyDeviceToHost, ctx->stream));
  MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return MTG_OK;
}

int mtg_last_kernel_ms(mtg_ctx* ctx, float* ms) {
  if (!ms) return MTG_ERR_INVALID_ARGUMENT;
  int n = 0;
  int rc = mtg_kernel_times(ctx, ms, 1, &n);
  if (rc == MTG_OK && n == 0) return set_error(ctx, MTG_ERR_INVALID_ARGUMENT, "no timed launch yet");
  return rc;
}

int mtg_enable_timing(mtg_ctx* ctx, int ring) {
  if (!ctx || ring < 0) return MTG_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(ctx->mu);
  MTG_HIP_TRY(ctx, hipSetDevice(ctx->device));
  MTG_HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  MTG_HIP_TRY(ctx, create_events(ctx, ring));
  return MTG_OK;
}

int mtg_kernel_times(mtg_ctx* ctx, float* ms, int n, int* n_out) {
  if (!ctx || !ms || n < 0 || !n_out) return MTG_ERR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(ctx->mu);
  MTG_HIP_TRY(ctx, hipSetDevice(ctx->device));
  const int64_t ring = (int64_t)ctx->ev_start.size();
  const int64_t have = std::min<int64_t>(ctx->launches, ring);
  const int64_t take = std::min<int64_t>(have, n);
  *n_out = 0;
  if (take == 0) return MTG_OK;
  const size_t newest = (size_t)((ctx->launches - 1) % ring);
  MTG_HIP_TRY(ctx, hipEventSynchronize(ctx->ev_stop[newest]));
  for (int64_t i = 0; i < take; ++i) {
    const size_t slot = (size_t)((ctx->launches - take + i) % ring);
    MTG_HIP_TRY(ctx, hipEventElapsedTime(&ms[i], ctx->ev_start[slot], ctx->ev_stop[slot]));
  }
  *n_out = (int)take;
  return MTG_OK;
}

}  // extern "C"

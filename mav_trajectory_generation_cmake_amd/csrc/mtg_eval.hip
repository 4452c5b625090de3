// mtg_eval.hip -- batched Trajectory::evaluateRange (src/trajectory.cpp:68-128).
//
// The reference advances its clock by repeated FP addition (acc += dt,
// tin += dt, tin -= T_i at a segment switch, :109-126), so the number of
// samples and every sample time depend on the sequential rounding.  Replaying
// that chain sample by sample costs ~80 cycles of FP64 latency per sample on
// gfx950 (scripts/micro/f64_latency.hip), ~0.6 M cycles per trajectory.
//
// These kernels reproduce it exactly without the chain.  While a positive
// double x stays inside one binade [2^e, 2^(e+1)), its grid spacing u is
// fixed, so fl(x + dt) = x + inc u with a constant integer inc = RNE(dt / u)
// (when dt / u is an exact half-integer, once the mantissa is even the tie
// always resolves to inc = q + (q & 1)).  The clock therefore splits into
// "runs": maximal ranges of samples on which tin and acc are both such
// progressions, ended by a binade crossing of either, a segment switch or
// t_end -- each found in closed form with integer arithmetic.  The step that
// ends a run is done as a real FP addition, so every state is the
// reference's.  A trajectory has ~10 runs per segment instead of ~750
// sequential steps; within a run every sample's (acc, tin) is
// (m + k inc) 2^E, which makes the evaluation fully parallel.  The segment
// polynomials use the reference's Horner form (Polynomial::evaluate,
// polynomial.h:138-151), multiply-then-add.
#include <float.h>

#include "mtg_device.h"

namespace mtg {

// Polynomial::base_coefficients_(n, i) = i!/(i-n)! (src/polynomial.cpp:140-155)
__device__ __forceinline__ double base_coeff(int n, int i) {
  if (i < n) return 0.0;
  double out = 1.0;
  for (int k = i - n + 1; k <= i; ++k) out *= (double)k;
  return out;
}

// Locate the start segment exactly as :82-105; returns false if t_start is out of range.
__device__ __forceinline__ bool range_start(const double* tms, int K, double t_start, int* seg,
                                            double* acc, double* tin) {
  double a = 0.0;
  int i = 0;
  for (i = 0; i < K; ++i) {
    a += tms[i];
    if (a > t_start) break;
  }
  if (t_start > a) return false;
  if (i >= K) i = K - 1;  // reference indexes segments_[K] here (UB); clamp to the last segment
  a -= tms[i];
  *seg = i;
  *acc = a;
  *tin = t_start - a;
  return true;
}

// x_k = (m + k inc) 2^E, k = 0, 1, ...: the values fl(x + dt) takes while x stays in its binade.
struct Prog {
  int64_t m, inc;
  int E;
};

constexpr int64_t kTwo53 = 9007199254740992LL;

// 1/den to a few ulp (v_rcp_f64 and one Newton step, multiply and subtract: not fused, so the
// kernel's only f64 FMAs stay the compiler's conversion idiom, tests/test_build.py), for
// floor_div_r: the two limits of a progression share its increment, so they share the reciprocal.
__device__ __forceinline__ double recip(int64_t den) {
#pragma clang fp contract(off)
  const double dd = (double)den;
  const double y = __builtin_amdgcn_rcp(dd);
  return y * (2.0 - dd * y);
}

// floor(num / den) for 0 <= num < 2^62, 0 < den < 2^62, given y = recip(den).  The estimate's error
// is ~q 2^-48 + 1, so one correction each way is exact for q < 2^45 (a run of 2^45 samples); the
// loops are the guard beyond that.  (Round 3 corrected by loops alone, each iteration a 64-bit
// multiply and an exec-mask round trip for the wave.)
__device__ __forceinline__ int64_t floor_div_r(int64_t num, int64_t den, double y) {
  double qd = (double)num * y;
  qd = qd < 4.0e18 ? qd : 4.0e18;
  int64_t q = (int64_t)qd;
  q = q < 0 ? 0 : q;
  int64_t r = num - q * den;
  if (r < 0) {
    --q;
    r += den;
  } else if (r >= den) {
    ++q;
    r -= den;
  }
  if (__builtin_expect(r < 0 || r >= den, 0)) {
    while (q > 0 && q * den > num) --q;
    while ((q + 1) * den <= num) ++q;
  }
  return q;
}

// (m + k inc) 2^E with m + k inc in [2^52, 2^53): the double is assembled from its bit fields
__device__ __forceinline__ double mant_exp(int64_t v, int E) {
  return __longlong_as_double(((int64_t)(E + 1075) << 52) | (v - (int64_t)(1ll << 52)));
}

// The progression of x under x <- fl(x + dt), if x is a normal positive double whose first step
// stays in its binade and is not an unresolved tie (odd mantissa).  Otherwise false: the caller
// takes one real step.
__device__ __forceinline__ bool progression(double x, double dt, Prog* p) {
  if (!(x > 0.0)) return false;
  const uint64_t bits = (uint64_t)__double_as_longlong(x);
  const int ex = (int)((bits >> 52) & 0x7FF);
  if (ex == 0 || ex == 0x7FF) return false;
  const int64_t m = (int64_t)((bits & ((1ull << 52) - 1)) | (1ull << 52));
  const int E = ex - 1075;
  const double f = __builtin_amdgcn_ldexp(dt, -E);  // dt / u, exact (power-of-two scaling)
  if (!(f < (double)(kTwo53 - m))) return false;     // the first step leaves the binade
  const double q = __builtin_floor(f);
  const double phi = f - q;
  const int64_t qi = (int64_t)q;
  int64_t inc;
  if (phi < 0.5) {
    inc = qi;
  } else if (phi > 0.5) {
    inc = qi + 1;
  } else {
    if (m & 1) return false;  // tie from an odd mantissa: one real step makes it even
    inc = qi + (qi & 1);
  }
  if (inc <= 0) return false;
  p->m = m;
  p->inc = inc;
  p->E = E;
  return true;
}

__device__ __forceinline__ double prog_value(const Prog& p, int64_t k) { return mant_exp(p.m + k * p.inc, p.E); }

constexpr int64_t kNoLimit = (int64_t)1 << 62;

// One run of the clock: samples n0 .. n0+L-1 at tin = prog_value(t, k), acc = prog_value(a, k)
// (L == 1 and single: the plain doubles tin0 / acc0), all in segment seg.
struct Run {
  int64_t n0, L;
  Prog t, a;
  double tin0, acc0;
  int seg;
  bool single;
};

// number of k >= 0 with m + k inc <= lim (lim given as a double, exact if < 2^62, else no limit),
// given y = recip(p.inc)
__device__ __forceinline__ int64_t run_len_le_r(const Prog& p, double lim_scaled, double y) {
  if (!(lim_scaled < 4.0e18)) return kNoLimit;
  const int64_t lim = (int64_t)lim_scaled;
  if (lim < p.m) return 0;
  return floor_div_r(lim - p.m, p.inc, y) + 1;
}

// The reference's clock (src/trajectory.cpp:86-127), advanced run by run.
//
// A run ends where the first of four limits is reached: tin leaves its binade, tin > T_i, acc leaves
// its binade, acc >= t_end.  The clock is one lane's serial chain, and the lanes of a wave run the
// union of their paths, so every call of next() does the same work on every lane: one run, then the
// reference's end-of-step checks -- acc >= t_end, and the segment switches (tin > T_i: tin -= T_i)
// -- folded into the same call rather than taken as a loop iteration of their own, which cost the
// whole wave a second run iteration whenever any of its lanes switched (round 3).  (Carrying the
// progressions from run to run instead of re-deriving them saves no time for the same reason: some
// lane of the wave re-derives each of them at almost every run.)
struct Clock {
  const double* T;
  int K;
  double dt, t_end;
  double acc, tin, Ti;
  int seg;
  int64_t n;
  bool done;

  // the reference's checks before a sample: stop at t_end, switch segments while tin > T_i
  __device__ __forceinline__ void settle() {
    if (!(acc < t_end)) {
      done = true;
      return;
    }
    while (tin > Ti) {  // segment switch: no sample, acc unchanged
      tin = tin - Ti;
      if (++seg >= K) {
        done = true;
        return;
      }
      Ti = T[seg];
    }
  }

  __device__ __forceinline__ void init(const double* tms, int K_, double t_start, double t_end_, double dt_) {
    T = tms;
    K = K_;
    dt = dt_;
    t_end = t_end_;
    n = 0;
    done = !range_start(tms, K, t_start, &seg, &acc, &tin);
    Ti = done ? 0.0 : T[seg];
    if (!done) settle();
  }

  // next run into *r; false when the clock has stopped
  __device__ __forceinline__ bool next(Run* r) {
    if (done) return false;
    r->n0 = n;
    r->seg = seg;
    r->tin0 = tin;
    r->acc0 = acc;
    Prog pt, pa;
    int64_t L = 1;
    r->single = true;
    if (progression(tin, dt, &pt) && progression(acc, dt, &pa)) {
      const double yt = recip(pt.inc), ya = recip(pa.inc);
      int64_t lim = floor_div_r(kTwo53 - 1 - pt.m, pt.inc, yt) + 1;                         // tin binade
      lim = min(lim, floor_div_r(kTwo53 - 1 - pa.m, pa.inc, ya) + 1);                         // acc binade
      lim = min(lim, run_len_le_r(pt, __builtin_amdgcn_ldexp(Ti, -pt.E), yt));               // tin <= T_i
      const double q = __builtin_amdgcn_ldexp(t_end, -pa.E);                                 // acc < t_end
      if (q < 4.0e18) lim = min(lim, run_len_le_r(pa, __builtin_ceil(q) - 1.0, ya));
      L = lim < 1 ? 1 : lim;
      r->t = pt;
      r->a = pa;
      r->single = false;
      if (L > 1) {  // state at the run's last sample, exactly
        tin = prog_value(pt, L - 1);
        acc = prog_value(pa, L - 1);
      }
    }
    r->L = L;
    n += L;
    tin += dt;  // the step after the run's last sample, as the reference takes it
    acc += dt;
    settle();
    return true;
  }
};

// A run as stored in the HBM run table (eval_runs_kernel -> eval_range_kernel), 64 B.  Its length is
// the next run's n0 less its own (the last stored run ends at RunHead::n); segs = 2 seg + single.
// The tin lane of eval_runs_kernel's lane pair writes bytes 0-31 and 56-61 (n0, tm, ti, tin0, segs,
// tE), the acc lane 32-55 and 62-63 (am, ai, acc0, aE).
struct RunRec {
  int64_t n0, tm, ti;
  double tin0;
  int64_t am, ai;
  double acc0;
  int32_t segs;
  int16_t tE, aE;
};
static_assert(sizeof(RunRec) == 64, "RunRec is one 64-B scalar load");

// Per trajectory: how many runs the table holds and, when the clock had not stopped by then, its
// state after them (the eval wave resumes the clock there).
struct RunHead {
  int64_t nruns, n;
  double acc, tin, Ti;
  int32_t seg, done;
};

// The other lane of a lane pair (2i, 2i + 1): DPP quad_perm [1, 0, 3, 2], no LDS.
__device__ __forceinline__ int pair_swap(int v) { return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int64_t pair_swap(int64_t v) {
  const int lo = pair_swap((int)(uint32_t)v), hi = pair_swap((int)(v >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
__device__ __forceinline__ double pair_swap(double v) {
  return __builtin_bit_cast(double, pair_swap(__builtin_bit_cast(int64_t, v)));
}

// The reference's clock on a lane pair: the even lane carries tin (and the segment), the odd lane
// acc.  A run's two progressions and their limits -- tin's binade and T_i, acc's binade and t_end
// -- are each one lane's work, and the lanes exchange only whether they have a progression and
// their limit (DPP), so a run's serial chain is half of Clock::next's.  The clock is the run
// kernels' critical path: one trajectory's ~110 runs back to back, one wave per SIMD.  Every
// shuffle is executed by both lanes of a pair (a pair stops together).
struct PairClock {
  const double* T;
  int K;
  double dt, t_end;
  double x;   // tin (even lane) or acc (odd lane)
  double Ti;  // (even lane)
  int seg;    // (even lane)
  int64_t n;
  bool done, odd;

  // the reference's checks before a sample (Clock::settle): the odd lane tests acc < t_end, then
  // the even lane switches segments while tin > T_i
  __device__ __forceinline__ void settle() {
    // (each pair_swap is evaluated unconditionally: a lane that skipped it would leave its partner
    // reading an inactive lane, and the pair would fall out of step)
    bool stop = done || (odd && !(x < t_end));
    const bool other = pair_swap((int)stop) != 0;
    stop = stop || other;
    if (!stop && !odd) {
      while (x > Ti) {
        x = x - Ti;
        if (++seg >= K) {
          stop = true;
          break;
        }
        Ti = T[seg];
      }
    }
    const bool other2 = pair_swap((int)stop) != 0;
    done = stop || other2;
  }

  __device__ __forceinline__ void init(const double* tms, int K_, double t_start, double t_end_, double dt_, bool odd_,
                                       bool valid) {
    T = tms;
    K = K_;
    dt = dt_;
    t_end = t_end_;
    odd = odd_;
    n = 0;
    double acc = 0.0, tin = 0.0;
    seg = 0;
    done = !(valid && range_start(tms, K, t_start, &seg, &acc, &tin));
    x = odd ? acc : tin;
    Ti = done ? 0.0 : T[seg];
    settle();
  }

  // the next run, written to *w (this lane's half) if w; false when the clock has stopped
  __device__ __forceinline__ bool next(RunRec* w) {
    if (done) return false;
    const int64_t n0 = n;
    const double x0 = x;
    const int seg0 = seg;
    Prog p;
    const bool ok = progression(x, dt, &p);
    int64_t lim = kNoLimit;
    if (ok) {
      const double y = recip(p.inc);
      lim = floor_div_r(kTwo53 - 1 - p.m, p.inc, y) + 1;  // the binade
      if (!odd) {
        lim = min(lim, run_len_le_r(p, __builtin_amdgcn_ldexp(Ti, -p.E), y));  // tin <= T_i
      } else {
        const double q = __builtin_amdgcn_ldexp(t_end, -p.E);  // acc < t_end
        if (q < 4.0e18) lim = min(lim, run_len_le_r(p, __builtin_ceil(q) - 1.0, y));
      }
    }
    const bool both = pair_swap((int)ok) != 0 && ok;
    const int64_t lim2 = pair_swap(lim);
    int64_t L = 1;
    if (both) {
      const int64_t m = min(lim, lim2);
      L = m < 1 ? 1 : m;
      if (L > 1) x = prog_value(p, L - 1);  // the run's last sample, exactly
    }
    n += L;
    x += dt;  // the step after it, as the reference takes it
    settle();
    if (w) {
      if (!odd) {
        w->n0 = n0;
        w->tm = p.m;
        w->ti = p.inc;
        w->tin0 = x0;
        w->segs = 2 * seg0 + (both ? 0 : 1);
        w->tE = (int16_t)p.E;
      } else {
        w->am = p.m;
        w->ai = p.inc;
        w->acc0 = x0;
        w->aE = (int16_t)p.E;
      }
    }
    return true;
  }
};

// Trajectories per block (one wave) of the clock kernels: a lane pair each.
constexpr int kPairTraj = 32;

// The segment times of the wave's 32 trajectories, staged in LDS (LT) when they fit kClockLdsK per
// trajectory.  Read from global memory inside the clock loop, each segment switch's load made the
// compiler wait for vmcnt(0) at the next run -- which also waits for every run-table store the
// wave has in flight, one store round trip per run.  LDS reads count on lgkmcnt only.
constexpr int kClockLdsK = 256;

template <bool LT>
__device__ __forceinline__ const double* clock_times(const double* times, int K, int64_t B, int lane) {
  const int64_t b0 = (int64_t)blockIdx.x * kPairTraj;
  const int64_t b = b0 + (lane >> 1);
  if constexpr (LT) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int nv = (int)(B - b0 < kPairTraj ? B - b0 : kPairTraj);
    const double* src = times + b0 * K;
    for (int j = lane; j < nv * K; j += 64) lds[j] = src[j];
    __syncthreads();  // (one wave)
    return lds + (b < B ? (int)(b - b0) : 0) * K;
  } else {
    return times + (b < B ? b : 0) * K;
  }
}

template <bool LT>
__global__ __launch_bounds__(64) void eval_count_kernel(int K, int64_t B, const double* times, double t_start,
                                                        double t_end, double dt, int64_t* counts) {
  const int lane = threadIdx.x;
  const int64_t b = (int64_t)blockIdx.x * kPairTraj + (lane >> 1);
  const bool valid = b < B;
  PairClock ck;
  ck.init(clock_times<LT>(times, K, B, lane), K, t_start, t_end, dt, lane & 1, valid);
  while (ck.next(nullptr)) {
  }
  if (valid && !(lane & 1)) counts[b] = ck.n;
}

// The clock, a lane pair per trajectory, writing its first `cap` runs to the run table.  The clock
// is a serial chain per trajectory; run here, 32 trajectories share a wave, where the eval kernel's
// lane 0 would run it alone while its wave waits.  (Round 3 ran one lane per trajectory: the run
// arithmetic of both progressions on one lane, 0.143 ms at 1e4.  16 or 32 trajectories per wave
// with one lane each measured slower than 64: 0.155 -> 0.205 / 0.166 ms.)
//
// With `counts` (the one-call evaluateRange, mtg_evaluate_range_batch_full) the kernel also finishes
// each clock to get the trajectory's sample count -- the count kernel's work, without running the
// clock twice -- and, per 32-trajectory block (one wave), writes the exclusive prefix sum of the
// counts inside the block to offs[b] and the block's total to bsum[block]: the first level of the
// device-side offsets (eval_scan_kernel, then the eval kernel adds the block's offset).
template <bool LT>
__global__ __launch_bounds__(64) void eval_runs_kernel(int K, int64_t B, const double* times, double t_start,
                                                       double t_end, double dt, int cap, RunHead* heads, RunRec* runs,
                                                       int64_t* counts, int64_t* offs, int64_t* bsum) {
  const int lane = threadIdx.x;
  const bool odd = lane & 1;
  const int64_t b = (int64_t)blockIdx.x * kPairTraj + (lane >> 1);
  const bool valid = b < B;
  PairClock ck;
  ck.init(clock_times<LT>(times, K, B, lane), K, t_start, t_end, dt, odd, valid);
  RunRec* rr = runs + (valid ? b : 0) * (int64_t)cap;
  int64_t nr = 0;
  while (nr < cap && ck.next(rr + nr)) ++nr;
  const double acc = pair_swap(ck.x);  // (the even lane's head needs acc)
  if (valid && !odd) {
    RunHead h;
    h.nruns = nr;
    h.n = ck.n;
    h.acc = acc;
    h.tin = ck.x;
    h.Ti = ck.Ti;
    h.seg = ck.seg;
    h.done = ck.done;
    heads[b] = h;
  }
  if (!counts) return;
  while (ck.next(nullptr)) {  // the rest of a clock longer than the table: counted only
  }
  const int64_t cnt = valid && !odd ? ck.n : 0;
  if (valid && !odd) counts[b] = cnt;
  // exclusive prefix of the wave's counts (odd lanes and lanes past B count 0) and the block total
  int64_t incl = cnt;
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const int64_t o = __shfl_up(incl, m, 64);
    if (lane >= m) incl += o;
  }
  if (valid && !odd) offs[b] = incl - cnt;
  if (lane == 63) bsum[blockIdx.x] = incl;
}

// Second level of the offsets: one block scans the per-block totals in place (exclusive) and writes
// the grand total.  nb = ceil(B / kPairTraj) entries (one per 32-trajectory block of the clock
// kernel); each thread takes a contiguous chunk.
constexpr int kScanThreads = 1024;
__global__ __launch_bounds__(kScanThreads) void eval_scan_kernel(int64_t nb, int64_t* bsum, int64_t* total) {
  __shared__ int64_t part[kScanThreads];
  const int t = threadIdx.x;
  const int64_t per = (nb + kScanThreads - 1) / kScanThreads;
  const int64_t i0 = (int64_t)t * per < nb ? (int64_t)t * per : nb, i1 = i0 + per < nb ? i0 + per : nb;
  int64_t s = 0;
  for (int64_t i = i0; i < i1; ++i) s += bsum[i];
  part[t] = s;
  __syncthreads();
  for (int m = 1; m < kScanThreads; m <<= 1) {  // inclusive scan of the chunk sums
    const int64_t o = t >= m ? part[t - m] : 0;
    __syncthreads();
    part[t] += o;
    __syncthreads();
  }
  int64_t run = part[t] - s;  // exclusive prefix of this chunk
  for (int64_t i = i0; i < i1; ++i) {
    const int64_t v = bsum[i];
    bsum[i] = run;
    run += v;
  }
  if (t == kScanThreads - 1) *total = part[t];
}

// Runs per round of the LDS table (from the run table, or built by lane 0), consumed by the wave.
constexpr int kRuns = 32;
constexpr int kEvalThreads = 64;

// (A run's length is the next run's n0 less its own.  Config 2, K = 10, D = 3, N = 10: this table
// 2.3 KB + the Horner terms 2.4 KB + the staged block 3 KB = 7.7 KB per wave, so 20 waves -- 5 per
// SIMD, amdgpu_waves_per_eu below -- fit in a CU's 160 KB.)
struct RunLds {  // structure of arrays in LDS
  int64_t n0[kRuns], tm[kRuns], ti[kRuns], am[kRuns], ai[kRuns];
  double tin0[kRuns], acc0[kRuns];
  int tE[kRuns], aE[kRuns], seg[kRuns], single[kRuns];
};

// Whether a trajectory is eval_range_kernel<..., ST = true>'s: its whole clock is in the run table
// (the run kernel finished it) and its rows are addressable with 32-bit byte offsets.
__device__ __forceinline__ bool stored_whole(const RunHead& h, int64_t n_total, int D) {
  return h.done != 0 && n_total * (int64_t)(D * 8) < (int64_t)kBufOOB;
}

// One wave per trajectory: lane 0 turns the clock into runs (a few tens per segment), all lanes
// evaluate the runs' samples -- consecutive samples on consecutive lanes -- with the coefficients
// staged in LDS.
// DER >= 0: the derivative order at compile time (0..4, the common ones); DER < 0: `derivative`.
// DD > 0: D at compile time (the sample loop takes kSpl samples per lane per block); 0: D at run time.
// ST: only the trajectories whose whole clock is in the run table (stored_whole), with the D = DD
// sample loop alone: no clock on lane 0 and no run-time-D loop in the kernel, which leaves it the
// registers of the sample loop only (the one-call evaluateRange; a second launch, ST = false with
// `rest`, takes the others).
constexpr int kSpl = 2;
constexpr int kEvalWaves = 5;  // waves per SIMD the stored-run (ST) kernel's registers are built for
template <int N, int DER, int DD, bool ST>
__global__ __launch_bounds__(kEvalThreads) __attribute__((amdgpu_waves_per_eu(ST ? kEvalWaves : 4))) void eval_range_kernel(int D, int K, const double* coeffs,
                                                                  const double* times, double t_start, double t_end,
                                                                  double dt, int derivative, const int64_t* counts,
                                                                  const int64_t* offsets, double* out,
                                                                  double* sample_times, int cap,
                                                                  const RunHead* heads, const RunRec* runs,
                                                                  const int64_t* boff, int64_t* offsets_out,
                                                                  int64_t capacity, const int64_t* total, bool rest) {
  // HIP defaults to -ffp-contract=fast-honor-pragmas: without this pragma the Horner step below
  // becomes an FMA (v_fmac_f64) and differs from the reference in the last bit.
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t n_total = counts[b];
  if constexpr (ST) {
    if (!stored_whole(heads[b], n_total, D)) return;
  } else {
    if (rest && stored_whole(heads[b], n_total, D)) return;  // (the stored-run launch has taken it)
  }
  // offsets: given (offsets[b]), or device-side (the in-block prefix offsets[b] + the block's offset)
  const int64_t base = boff ? offsets[b] + boff[b / kPairTraj] : offsets[b];
  if (boff && lane == 0) offsets_out[b] = base;
  // (past the caller's capacity -- this trajectory's rows, or the call's total when it is known on the
  // device: then nothing at all is written)
  if (n_total <= 0 || base + n_total > capacity || (total && *total > capacity)) return;
  RunLds* rt = reinterpret_cast<RunLds*>(lds);
  double* cf = reinterpret_cast<double*>(rt + 1);  // [K][D][N]
  double* ob = cf + K * D * N;                     // [kEvalThreads][D] output block
  // The D-at-compile-time sample loop stores through buffer resources over this trajectory's rows and
  // sample times, addressed by 32-bit byte offsets (a trajectory with under 2 GiB of rows; longer
  // ones take the run-time-D loop), with 16-B pieces when `out` is 16-B aligned.
  const bool fast = ST || (DD > 0 && n_total * (int64_t)(D * 8) < (int64_t)kBufOOB);
  const bool al16 = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
  const __amdgpu_buffer_rsrc_t ro = buf_rsrc(out + base * D, fast ? (uint32_t)(n_total * D * 8) : 0u);
  const __amdgpu_buffer_rsrc_t rs =
      buf_rsrc(sample_times ? sample_times + base : out, fast && sample_times ? (uint32_t)(n_total * 8) : 0u);
  const double* cb = coeffs + b * (int64_t)K * D * N;
  if (DER >= 0) derivative = DER;
  // the Horner terms base_coefficients_(derivative, j) * coefficients_[j] (polynomial.h:143-148) do
  // not depend on t: formed once per coefficient here, with the same rounding as the reference's
  // per-sample products
  for (int i = lane; i < K * D * N; i += kEvalThreads) cf[i] = base_coeff(derivative, i % N) * cb[i];
  Clock ck;
  int64_t stored = 0, next_run = 0, stored_end = 0;  // runs in the HBM table, runs taken from it, where they end
  const RunRec* rr = runs ? runs + b * (int64_t)cap : nullptr;
  if (heads) {
    const RunHead h = heads[b];
    stored = h.nruns;
    stored_end = h.n;
    if (!ST && lane == 0) {  // resume the clock after the stored runs
      ck.T = times + b * K;
      ck.K = K;
      ck.dt = dt;
      ck.t_end = t_end;
      ck.acc = h.acc;
      ck.tin = h.tin;
      ck.Ti = h.Ti;
      ck.seg = h.seg;
      ck.n = h.n;
      ck.done = h.done != 0;
    }
  } else if (!ST && lane == 0) {
    ck.init(times + b * K, K, t_start, t_end, dt);
  }
  __shared__ int s_nr;
  __shared__ int64_t s_end;
  for (;;) {
    if (next_run < stored) {  // a round from the run table: one run per lane
      const int nr = (int)(stored - next_run < kRuns ? stored - next_run : kRuns);
      if (lane < nr) {
        const RunRec w = rr[next_run + lane];
        rt->n0[lane] = w.n0;
        rt->tm[lane] = w.tm;
        rt->ti[lane] = w.ti;
        rt->tE[lane] = w.tE;
        rt->am[lane] = w.am;
        rt->ai[lane] = w.ai;
        rt->aE[lane] = w.aE;
        rt->tin0[lane] = w.tin0;
        rt->acc0[lane] = w.acc0;
        rt->seg[lane] = w.segs >> 1;
        rt->single[lane] = w.segs & 1;
        if (lane == nr - 1) s_end = next_run + nr < stored ? rr[next_run + nr].n0 : stored_end;
      }
      if (lane == 0) s_nr = nr;
      next_run += nr;
    } else if (ST) {
      if (lane == 0) s_nr = 0;  // (the table held the whole clock)
    } else if (lane == 0) {
      int nr = 0;
      Run r;
      while (nr < kRuns && ck.next(&r)) {
        rt->n0[nr] = r.n0;
        rt->tm[nr] = r.t.m;
        rt->ti[nr] = r.t.inc;
        rt->tE[nr] = r.t.E;
        rt->am[nr] = r.a.m;
        rt->ai[nr] = r.a.inc;
        rt->aE[nr] = r.a.E;
        rt->tin0[nr] = r.tin0;
        rt->acc0[nr] = r.acc0;
        rt->seg[nr] = r.seg;
        rt->single[nr] = r.single;
        ++nr;
      }
      s_nr = nr;
      s_end = ck.n;
    }
    lds_fence();  // (one wave per block: the table is complete for every lane)
    const int nr = s_nr;
    if (nr == 0) break;
    const int64_t first = rt->n0[0], end = s_end < n_total ? s_end : n_total;
    int ri = 0;
    if (ST || (DD > 0 && fast)) {
      // D at compile time: each lane takes kSpl samples per block (n = nb + s 64 + lane), and their
      // kSpl D Horner chains are independent, so they interleave instead of running one dimension
      // after the other; the staged rows are read back in one batch before the stores.
      constexpr int kBlk = kSpl * kEvalThreads;
      constexpr int DDc = DD > 0 ? DD : 1;
      // 16-B row pieces: a full block's kBlk DD doubles are kBlk DD / 128 pieces per lane
      constexpr int P16 = kBlk * DDc / (2 * kEvalThreads);
      int64_t nxt = ri + 1 < nr ? rt->n0[ri + 1] : INT64_MAX;  // the next run's first sample
      double cc[DDc * N];  // the cached segment's Horner terms (wave-uniform: SGPRs)
      int cseg = -1;
      for (int64_t nb = first; nb < end;) {
        // blocks start where the rows are 16-B aligned in `out` (an odd D: (base + nb) even), so a
        // full block leaves in 16-B pieces; the round's first block may be one sample short
        int cnt = (int)(end - nb < kBlk ? end - nb : kBlk);
        if ((DDc & 1) && (((base + nb) & 1) != 0) && cnt == kBlk) cnt = kBlk - 1;
        double tv[kSpl];
        const double* cs[kSpl];
        int sg[kSpl];
#pragma unroll
        for (int s = 0; s < kSpl; ++s) {
          const int64_t n = nb + s * kEvalThreads + lane;
          const bool have = s * kEvalThreads + lane < cnt;
          while (have && nxt <= n) {
            ++ri;
            nxt = ri + 1 < nr ? rt->n0[ri + 1] : INT64_MAX;
          }
          const int64_t k = n - rt->n0[ri];
          double t, a;
          if (rt->single[ri]) {
            t = rt->tin0[ri];
            a = rt->acc0[ri];
          } else {
            t = mant_exp(rt->tm[ri] + k * rt->ti[ri], rt->tE[ri]);
            a = sample_times ? mant_exp(rt->am[ri] + k * rt->ai[ri], rt->aE[ri]) : 0.0;
          }
          tv[s] = t;
          sg[s] = rt->seg[ri];
          cs[s] = cf + (sg[s] * DDc) * N;
          if (sample_times)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, a), rs, have ? (uint32_t)(n * 8) : kBufOOB, 0, 0);
        }
        double v[kSpl][DDc];
        // Usually the whole block lies in one segment (a segment has ~750 samples at dt = 0.01): its
        // Horner terms then come from SGPRs (read from LDS only when the wave's segment changes),
        // which leaves the VGPRs to the samples.  Per-lane LDS reads of every coefficient for every
        // sample made the CU's LDS bandwidth the limit (~30 16-B reads per lane per block).
        const int sg0 = __builtin_amdgcn_readfirstlane(sg[0]);
        bool same = true;
#pragma unroll
        for (int s = 0; s < kSpl; ++s) same = same && sg[s] == sg0;
        if (__builtin_amdgcn_ballot_w64(!same) == 0) {
          if (sg0 != cseg) {
            const double* c0 = cf + (sg0 * DDc) * N;
#pragma unroll
            for (int i = 0; i < DDc * N; ++i) {
              const uint64_t w = __builtin_bit_cast(uint64_t, c0[i]);
              const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(w >> 32));
              const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)w);
              cc[i] = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
            }
            cseg = sg0;
          }
#pragma unroll
          for (int s = 0; s < kSpl; ++s)
#pragma unroll
            for (int d = 0; d < DDc; ++d) v[s][d] = derivative < N ? cc[d * N + N - 1] : 0.0;
          if (derivative < N) {
#pragma unroll
            for (int j = N - 2; j >= 0; --j) {
              if (DER >= 0 ? j >= DER : j >= derivative) {
#pragma unroll
                for (int s = 0; s < kSpl; ++s)
#pragma unroll
                  for (int d = 0; d < DDc; ++d) {
                    v[s][d] = v[s][d] * tv[s];
                    v[s][d] = v[s][d] + cc[d * N + j];
                  }
              }
            }
          }
        } else {
#pragma unroll
          for (int s = 0; s < kSpl; ++s)
#pragma unroll
            for (int d = 0; d < DDc; ++d) v[s][d] = derivative < N ? cs[s][d * N + N - 1] : 0.0;
          if (derivative < N) {
#pragma unroll
            for (int j = N - 2; j >= 0; --j) {
              if (DER >= 0 ? j >= DER : j >= derivative) {
#pragma unroll
                for (int s = 0; s < kSpl; ++s)
#pragma unroll
                  for (int d = 0; d < DDc; ++d) {
                    v[s][d] = v[s][d] * tv[s];
                    v[s][d] = v[s][d] + cs[s][d * N + j];
                  }
              }
            }
          }
        }
#pragma unroll
        for (int s = 0; s < kSpl; ++s)
#pragma unroll
          for (int d = 0; d < DDc; ++d) ob[(s * kEvalThreads + lane) * DDc + d] = v[s][d];
        lds_fence();  // one wave per block: the staged rows are complete
        const uint32_t o0 = (uint32_t)(nb * DDc * 8);  // the block's first row, bytes into the trajectory's rows
        if (cnt == kBlk && al16) {  // whole 16-B pieces, 1 KiB per store instruction
          dvec2 w[P16];
#pragma unroll
          for (int u = 0; u < P16; ++u) w[u] = *reinterpret_cast<const dvec2*>(ob + 2 * (u * kEvalThreads + lane));
          lds_fence();  // (read before the next block overwrites them)
#pragma unroll
          for (int u = 0; u < P16; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, w[u]), ro, o0 + (uint32_t)(u * kEvalThreads + lane) * 16, 0, 0);
        } else {
          double w[kSpl * DDc];
#pragma unroll
          for (int u = 0; u < kSpl * DDc; ++u) w[u] = ob[u * kEvalThreads + lane];
          lds_fence();
#pragma unroll
          for (int u = 0; u < kSpl * DDc; ++u)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, w[u]), ro,
                                                  u * kEvalThreads + lane < cnt * DDc ? o0 + (uint32_t)(u * kEvalThreads + lane) * 8 : kBufOOB, 0, 0);
        }
        nb += cnt;
      }
      if (end >= n_total) break;
      lds_fence();  // the run table is refilled next (one wave: no barrier, no wait on the stores)
      continue;
    }
    for (int64_t nb = first; nb < end; nb += kEvalThreads) {
      const int64_t n = nb + lane;
      const int cnt = (int)(end - nb < kEvalThreads ? end - nb : kEvalThreads);
      if (n < end) {
        while (ri + 1 < nr && rt->n0[ri + 1] <= n) ++ri;
        const int64_t k = n - rt->n0[ri];
        double t, a;
        if (rt->single[ri]) {
          t = rt->tin0[ri];
          a = rt->acc0[ri];
        } else {
          t = mant_exp(rt->tm[ri] + k * rt->ti[ri], rt->tE[ri]);
          a = mant_exp(rt->am[ri] + k * rt->ai[ri], rt->aE[ri]);
        }
        const double* cs = cf + (rt->seg[ri] * D) * N;
        for (int d = 0; d < D; ++d) {
          double v = 0.0;
          if (derivative < N) {
            const double* c = cs + d * N;
            v = c[N - 1];
#pragma unroll
            for (int j = N - 2; j >= 0; --j) {
              if (DER >= 0 ? j >= DER : j >= derivative) {
                v = v * t;
                v = v + c[j];
              }
            }
          }
          ob[lane * D + d] = v;
        }
        if (sample_times) sample_times[base + n] = a;
      }
      lds_fence();
      // the block's rows are contiguous in out: write them with consecutive lanes
      double* dst = out + (base + nb) * D;
      for (int i = lane; i < cnt * D; i += kEvalThreads) dst[i] = ob[i];
      lds_fence();
    }
    if (end >= n_total) break;
  }
}

// The stored-run sample loop for D = 3 as a producer / consumer pair (MTG_EVAL_PC): a block of two
// waves per trajectory, wave 0 evaluating the samples block by block into one of two LDS slots,
// wave 1 storing the other slot's rows and sample times.  In the one-wave kernel the same wave
// computed and stored, and a store that could not issue (the memory queue full) held up its
// compute; the kernel took ~0.63 ms where its compute alone took ~0.39 and its stores alone ~0.44.
// The two waves meet at one s_barrier per block; the barrier waits only for LDS (the store wave's
// global stores stay in flight).  Samples, rows and their order are the one-wave kernel's exactly.
constexpr int kEvalPcWaves = 5;  // waves per SIMD the producer / consumer kernel is built for
struct PcSlot {
  double v[kSpl * kEvalThreads * 3];  // the block's rows, sample-major
  double ts[kSpl * kEvalThreads];     // its sample times
  int64_t nb;                         // its first sample (trajectory-relative)
  int cnt;                            // its samples; 0: the trajectory is done
  int pad;
};
static_assert(sizeof(PcSlot) % 16 == 0, "slots stay 16-B aligned");

// s_barrier after this wave's LDS accesses; unlike __syncthreads, no wait for its global stores
__device__ __forceinline__ void pc_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int N, int DER>
__global__ __launch_bounds__(2 * kEvalThreads) __attribute__((amdgpu_waves_per_eu(kEvalPcWaves))) void eval_range_pc_kernel(
    int K, const double* coeffs, int derivative, const int64_t* counts, const int64_t* offsets, double* out,
    double* sample_times, int cap, const RunHead* heads, const RunRec* runs, const int64_t* boff,
    int64_t* offsets_out, int64_t capacity, const int64_t* total) {
#pragma clang fp contract(off)
  constexpr int DD = 3;
  constexpr int kBlk = kSpl * kEvalThreads;
  constexpr int P16 = kBlk * DD / (2 * kEvalThreads);
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int64_t b = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t n_total = counts[b];
  const RunHead h = heads[b];
  if (!stored_whole(h, n_total, DD)) return;  // (the rest launch takes it)
  const int64_t base = boff ? offsets[b] + boff[b / kPairTraj] : offsets[b];
  if (boff && tid == 0) offsets_out[b] = base;
  if (n_total <= 0 || base + n_total > capacity || (total && *total > capacity)) return;
  RunLds* rt = reinterpret_cast<RunLds*>(lds);
  double* cf = reinterpret_cast<double*>(rt + 1);       // [K][3][N]
  PcSlot* slot = reinterpret_cast<PcSlot*>(cf + K * DD * N);  // [2]
  if (DER >= 0) derivative = DER;
  const double* cb = coeffs + b * (int64_t)K * DD * N;
  for (int i = tid; i < K * DD * N; i += 2 * kEvalThreads) cf[i] = base_coeff(derivative, i % N) * cb[i];
  __syncthreads();

  if (wave == 1) {  // ---- the store wave
    const bool al16 = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    const __amdgpu_buffer_rsrc_t ro = buf_rsrc(out + base * DD, (uint32_t)(n_total * DD * 8));
    const __amdgpu_buffer_rsrc_t rs =
        buf_rsrc(sample_times ? sample_times + base : out, sample_times ? (uint32_t)(n_total * 8) : 0u);
    for (int i = 0;; ++i) {
      pc_barrier();
      const PcSlot* sl = slot + (i & 1);
      const int cnt = sl->cnt;
      if (cnt == 0) break;
      const int64_t nb = sl->nb;
      double tv[kSpl];
#pragma unroll
      for (int q = 0; q < kSpl; ++q) tv[q] = sl->ts[q * kEvalThreads + lane];
      const uint32_t o0 = (uint32_t)(nb * DD * 8);
      if (cnt == kBlk && al16) {
        dvec2 w[P16];
#pragma unroll
        for (int u = 0; u < P16; ++u) w[u] = reinterpret_cast<const dvec2*>(sl->v)[u * kEvalThreads + lane];
        lds_fence();  // (read before the barrier lets the compute wave refill the slot)
#pragma unroll
        for (int u = 0; u < P16; ++u)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, w[u]), ro, o0 + (uint32_t)(u * kEvalThreads + lane) * 16, 0, 0);
      } else {
        double w[kSpl * DD];
#pragma unroll
        for (int u = 0; u < kSpl * DD; ++u) w[u] = sl->v[u * kEvalThreads + lane];
        lds_fence();
#pragma unroll
        for (int u = 0; u < kSpl * DD; ++u)
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, w[u]), ro,
                                                u * kEvalThreads + lane < cnt * DD ? o0 + (uint32_t)(u * kEvalThreads + lane) * 8 : kBufOOB, 0, 0);
      }
      if (sample_times) {
#pragma unroll
        for (int q = 0; q < kSpl; ++q)
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, tv[q]), rs,
                                                q * kEvalThreads + lane < cnt ? (uint32_t)((nb + q * kEvalThreads + lane) * 8) : kBufOOB, 0, 0);
      }
    }
    return;
  }

  // ---- the compute wave: the runs from the table, 32 per round; blocks of kBlk samples
  const RunRec* rr = runs + b * (int64_t)cap;
  const int64_t stored = h.nruns, stored_end = h.n;
  int64_t next_run = 0;
  int blk = 0;
  double cc[DD * N];  // the cached segment's Horner terms (wave-uniform: SGPRs)
  int cseg = -1;
  while (next_run < stored) {
    const int nr = (int)(stored - next_run < kRuns ? stored - next_run : kRuns);
    if (lane < nr) {
      const RunRec w = rr[next_run + lane];
      rt->n0[lane] = w.n0;
      rt->tm[lane] = w.tm;
      rt->ti[lane] = w.ti;
      rt->tE[lane] = w.tE;
      rt->am[lane] = w.am;
      rt->ai[lane] = w.ai;
      rt->aE[lane] = w.aE;
      rt->tin0[lane] = w.tin0;
      rt->acc0[lane] = w.acc0;
      rt->seg[lane] = w.segs >> 1;
      rt->single[lane] = w.segs & 1;
    }
    const int64_t round_end = next_run + nr < stored ? rr[next_run + nr].n0 : stored_end;
    next_run += nr;
    lds_fence();
    const int64_t first = rt->n0[0], end = round_end < n_total ? round_end : n_total;
    int ri = 0;
    int64_t nxt = ri + 1 < nr ? rt->n0[ri + 1] : INT64_MAX;
    for (int64_t nb = first; nb < end;) {
      int cnt = (int)(end - nb < kBlk ? end - nb : kBlk);
      if ((((base + nb) & 1) != 0) && cnt == kBlk) cnt = kBlk - 1;  // (rows 16-B aligned from the next block on)
      PcSlot* sl = slot + (blk & 1);
      double tv[kSpl];
      int sg[kSpl];
#pragma unroll
      for (int q = 0; q < kSpl; ++q) {
        const int64_t n = nb + q * kEvalThreads + lane;
        const bool have = q * kEvalThreads + lane < cnt;
        while (have && nxt <= n) {
          ++ri;
          nxt = ri + 1 < nr ? rt->n0[ri + 1] : INT64_MAX;
        }
        const int64_t k = n - rt->n0[ri];
        double t, a;
        if (rt->single[ri]) {
          t = rt->tin0[ri];
          a = rt->acc0[ri];
        } else {
          t = mant_exp(rt->tm[ri] + k * rt->ti[ri], rt->tE[ri]);
          a = sample_times ? mant_exp(rt->am[ri] + k * rt->ai[ri], rt->aE[ri]) : 0.0;
        }
        tv[q] = t;
        sg[q] = rt->seg[ri];
        sl->ts[q * kEvalThreads + lane] = a;
      }
      double v[kSpl][DD];
      const int sg0 = __builtin_amdgcn_readfirstlane(sg[0]);
      bool same = true;
#pragma unroll
      for (int q = 0; q < kSpl; ++q) same = same && sg[q] == sg0;
      if (__builtin_amdgcn_ballot_w64(!same) == 0) {
        if (sg0 != cseg) {
          const double* c0 = cf + (sg0 * DD) * N;
#pragma unroll
          for (int i = 0; i < DD * N; ++i) {
            const uint64_t w = __builtin_bit_cast(uint64_t, c0[i]);
            const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(w >> 32));
            const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)w);
            cc[i] = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
          }
          cseg = sg0;
        }
#pragma unroll
        for (int q = 0; q < kSpl; ++q)
#pragma unroll
          for (int d = 0; d < DD; ++d) v[q][d] = derivative < N ? cc[d * N + N - 1] : 0.0;
        if (derivative < N) {
#pragma unroll
          for (int j = N - 2; j >= 0; --j) {
            if (DER >= 0 ? j >= DER : j >= derivative) {
#pragma unroll
              for (int q = 0; q < kSpl; ++q)
#pragma unroll
                for (int d = 0; d < DD; ++d) {
                  v[q][d] = v[q][d] * tv[q];
                  v[q][d] = v[q][d] + cc[d * N + j];
                }
            }
          }
        }
      } else {
        const double* cs[kSpl];
#pragma unroll
        for (int q = 0; q < kSpl; ++q) cs[q] = cf + (sg[q] * DD) * N;
#pragma unroll
        for (int q = 0; q < kSpl; ++q)
#pragma unroll
          for (int d = 0; d < DD; ++d) v[q][d] = derivative < N ? cs[q][d * N + N - 1] : 0.0;
        if (derivative < N) {
#pragma unroll
          for (int j = N - 2; j >= 0; --j) {
            if (DER >= 0 ? j >= DER : j >= derivative) {
#pragma unroll
              for (int q = 0; q < kSpl; ++q)
#pragma unroll
                for (int d = 0; d < DD; ++d) {
                  v[q][d] = v[q][d] * tv[q];
                  v[q][d] = v[q][d] + cs[q][d * N + j];
                }
            }
          }
        }
      }
#pragma unroll
      for (int q = 0; q < kSpl; ++q)
#pragma unroll
        for (int d = 0; d < DD; ++d) sl->v[(q * kEvalThreads + lane) * DD + d] = v[q][d];
      if (lane == 0) {
        sl->nb = nb;
        sl->cnt = cnt;
      }
      pc_barrier();  // the slot to the store wave
      ++blk;
      nb += cnt;
    }
    if (end >= n_total) break;
  }
  if (lane == 0) slot[blk & 1].cnt = 0;  // done
  pc_barrier();
}

hipError_t launch_eval_count(int N, int D, int K, int64_t B, const double* times, double t_start,
                             double t_end, double dt, int64_t* counts, hipStream_t stream) {
  (void)N;
  (void)D;
  // one wave per 32 trajectories (a lane pair each); (256-thread blocks put the 1e4 clocks of config
  // 2 on 40 CUs: 0.163 -> 0.154 ms, round 2)
  const int64_t grid = (B + kPairTraj - 1) / kPairTraj;
  if (grid == 0) return hipSuccess;
  if (K <= kClockLdsK)
    launch_kernel(eval_count_kernel<true>, dim3((unsigned)grid), dim3(64), (uint32_t)(sizeof(double) * kPairTraj * K),
                  stream, K, B, times, t_start, t_end, dt, counts);
  else
    launch_kernel(eval_count_kernel<false>, dim3((unsigned)grid), dim3(64), 0, stream, K, B, times, t_start, t_end, dt,
                  counts);
  return hipGetLastError();
}

size_t eval_workspace_bytes(int K, int64_t B, int* cap) {
  // up to 256 runs per trajectory (config 2 has ~100-130: at 128 some trajectories overflowed to
  // the slow path, 0.793 -> 0.785 ms at 1e4), fewer for huge batches: the table is only written as
  // far as each trajectory's runs go and is capped at 2 GB; a trajectory with more runs than the
  // table holds continues on its eval wave's lane 0
  (void)K;
  int c = 256;
  while (c > 8 && (double)B * (c * sizeof(RunRec) + sizeof(RunHead)) > 2.0e9) c /= 2;
  *cap = c;
  return (size_t)B * (sizeof(RunHead) + (size_t)c * sizeof(RunRec));
}

size_t eval_full_workspace_bytes(int K, int64_t B, int* cap) {
  // the run table, then the per-block totals and the grand total
  return eval_workspace_bytes(K, B, cap) + sizeof(int64_t) * (size_t)((B + kPairTraj - 1) / kPairTraj + 1);
}

hipError_t launch_eval_runs_counts(int K, int64_t B, const double* times, double t_start, double t_end, double dt,
                                   int64_t* counts, int64_t* offsets, void* ws, int cap, int64_t* total,
                                   hipStream_t stream) {
  if (B == 0) return hipSuccess;
  RunHead* heads = static_cast<RunHead*>(ws);
  RunRec* runs = reinterpret_cast<RunRec*>(heads + B);
  int64_t* bsum = reinterpret_cast<int64_t*>(runs + (size_t)B * cap);
  const int64_t nb = (B + kPairTraj - 1) / kPairTraj;
  if (K <= kClockLdsK)
    launch_kernel(eval_runs_kernel<true>, dim3((unsigned)nb), dim3(64), (uint32_t)(sizeof(double) * kPairTraj * K),
                  stream, K, B, times, t_start, t_end, dt, cap, heads, runs, counts, offsets, bsum);
  else
    launch_kernel(eval_runs_kernel<false>, dim3((unsigned)nb), dim3(64), 0, stream, K, B, times, t_start, t_end, dt,
                  cap, heads, runs, counts, offsets, bsum);
  hipLaunchKernelGGL(eval_scan_kernel, dim3(1), dim3(kScanThreads), 0, stream, nb, bsum, total);
  return hipGetLastError();
}

hipError_t launch_eval_range(int N, int D, int K, int64_t B, const double* coeffs, const double* times,
                             double t_start, double t_end, double dt, int derivative, const int64_t* counts,
                             const int64_t* offsets, double* out, double* sample_times, void* ws, int cap,
                             hipStream_t stream, bool runs_ready, int64_t* offsets_out, int64_t capacity,
                             const int64_t* total) {
  if (B == 0) return hipSuccess;
  RunHead* heads = nullptr;
  RunRec* runs = nullptr;
  const int64_t* boff = nullptr;
  if (ws && cap > 0) {
    heads = static_cast<RunHead*>(ws);
    runs = reinterpret_cast<RunRec*>(heads + B);
    if (runs_ready) {  // launch_eval_runs_counts filled the table, the in-block offsets and the block offsets
      boff = reinterpret_cast<const int64_t*>(runs + (size_t)B * cap);
    } else {
      const dim3 g((unsigned)((B + kPairTraj - 1) / kPairTraj));
      if (K <= kClockLdsK)
        launch_kernel(eval_runs_kernel<true>, g, dim3(64), (uint32_t)(sizeof(double) * kPairTraj * K), stream, K, B,
                      times, t_start, t_end, dt, cap, heads, runs, (int64_t*)nullptr, (int64_t*)nullptr,
                      (int64_t*)nullptr);
      else
        launch_kernel(eval_runs_kernel<false>, g, dim3(64), 0, stream, K, B, times, t_start, t_end, dt, cap, heads,
                      runs, (int64_t*)nullptr, (int64_t*)nullptr, (int64_t*)nullptr);
    }
  }
  // D = 3 (every reference problem in 3-D) has its own kernels: the sample loop's dimensions unrolled
  const bool d3 = D == 3;
  // One block per trajectory.  (Splitting a trajectory's samples over 2 or 4 blocks, to shorten the
  // launch's tail, measured slower at 1e4 config-2 trajectories: 0.795 -> 0.80 / 0.855 ms; every
  // block reloads the run table and stages the coefficients.)
  const size_t lds = sizeof(RunLds) + sizeof(double) * ((size_t)K * D * N + (size_t)(d3 ? kSpl : 1) * kEvalThreads * D);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  const size_t lds_pc = sizeof(RunLds) + sizeof(double) * (size_t)K * 3 * N + 2 * sizeof(PcSlot);
  const bool pc = lds_pc <= 64 * 1024;  // (else the one-wave kernel)
  const dim3 grid((unsigned)B);
  // D = 3 with the run table: a stored-run launch takes every trajectory whose whole clock is in it
  // (the producer / consumer kernel, or the one-wave ST kernel when its LDS would not fit), and the
  // run-time-D kernel (rest) the others -- its blocks for the stored ones return at once
  const bool stored = heads != nullptr && d3;
#define MTG_EVAL_LAUNCH(NN, DER)                                                                                   \
  do {                                                                                                             \
    if (stored && pc) {                                                                                            \
      launch_kernel(eval_range_pc_kernel<NN, DER>, grid, dim3(2 * kEvalThreads), lds_pc, stream, K, coeffs,        \
                    derivative, counts, offsets, out, sample_times, cap, heads, runs, boff, offsets_out, capacity, \
                    total);                                                                                        \
      launch_kernel(eval_range_kernel<NN, DER, 0, false>, grid, dim3(kEvalThreads), lds, stream, D, K, coeffs,     \
                    times, t_start, t_end, dt, derivative, counts, offsets, out, sample_times, cap, heads, runs,  \
                    boff, offsets_out, capacity, total, true);                                                     \
    } else if (stored) {                                                                                           \
      launch_kernel(eval_range_kernel<NN, DER, 3, true>, grid, dim3(kEvalThreads), lds, stream, D, K, coeffs,      \
                    times, t_start, t_end, dt, derivative, counts, offsets, out, sample_times, cap, heads, runs,  \
                    boff, offsets_out, capacity, total, false);                                                    \
      launch_kernel(eval_range_kernel<NN, DER, 0, false>, grid, dim3(kEvalThreads), lds, stream, D, K, coeffs,     \
                    times, t_start, t_end, dt, derivative, counts, offsets, out, sample_times, cap, heads, runs,  \
                    boff, offsets_out, capacity, total, true);                                                     \
    } else if (d3) {                                                                                               \
      launch_kernel(eval_range_kernel<NN, DER, 3, false>, grid, dim3(kEvalThreads), lds, stream, D, K, coeffs,     \
                    times, t_start, t_end, dt, derivative, counts, offsets, out, sample_times, cap, heads, runs,  \
                    boff, offsets_out, capacity, total, false);                                                    \
    } else {                                                                                                       \
      launch_kernel(eval_range_kernel<NN, DER, 0, false>, grid, dim3(kEvalThreads), lds, stream, D, K, coeffs,     \
                    times, t_start, t_end, dt, derivative, counts, offsets, out, sample_times, cap, heads, runs,  \
                    boff, offsets_out, capacity, total, false);                                                    \
    }                                                                                                              \
  } while (0)
#define MTG_EVAL_CASE(NN)                 \
  case NN:                                \
    switch (derivative) {                 \
      case 0: MTG_EVAL_LAUNCH(NN, 0); break; \
      case 1: MTG_EVAL_LAUNCH(NN, 1); break; \
      case 2: MTG_EVAL_LAUNCH(NN, 2); break; \
      case 3: MTG_EVAL_LAUNCH(NN, 3); break; \
      case 4: MTG_EVAL_LAUNCH(NN, 4); break; \
      default: MTG_EVAL_LAUNCH(NN, -1); break; \
    }                                     \
    break;
  switch (N) {
    MTG_EVAL_CASE(2)
    MTG_EVAL_CASE(4)
    MTG_EVAL_CASE(6)
    MTG_EVAL_CASE(8)
    MTG_EVAL_CASE(10)
    MTG_EVAL_CASE(12)
    default: return hipErrorInvalidValue;
  }
#undef MTG_EVAL_CASE
#undef MTG_EVAL_LAUNCH
  return hipGetLastError();
}

}  // namespace mtg

/* Negative control of the TSan run (tests/test_sanitizers.py): the race class that reached the
 * smoke in round 3 -- a table filled lazily by whichever OpenMP thread gets there first while the
 * others read it.  The TSan build of this file must report a data race; if it does not, the
 * sanitizer setup (compiler, OpenMP runtime, archer) cannot see that class and the driver's clean
 * run proves nothing. */
#include <stdio.h>
#include <omp.h>

static double table[64];
static int table_ready = 0;

static double lookup(int i) {
  if (!table_ready) {
    for (int k = 0; k < 64; ++k) table[k] = k * 0.5;
    table_ready = 1;
  }
  return table[i & 63];
}

int main(void) {
  double acc = 0.0;
  omp_set_num_threads(8);
#pragma omp parallel for reduction(+ : acc) schedule(static, 1)
  for (int i = 0; i < 4096; ++i) acc += lookup(i);
  printf("%f\n", acc);
  return 0;
}

// Microbenchmark: cost of taken vs not-taken uniform scalar branches on gfx950 (inline asm
// so the compiler cannot if-convert).  Per loop iteration, 8 blocks of:
//   mode 0: s_cmp + s_cbranch (TAKEN, skips the v_add)
//   mode 1: s_cmp + s_cbranch (not taken) + v_add
//   mode 2: s_cmp + v_add (no branch)
#include <hip/hip_runtime.h>
#include <cstdio>

#define BLK_BR "s_cmp_eq_u32 %1, 0\n s_cbranch_scc1 1f\n v_add_f32 %0, 1.0, %0\n1:\n"
#define BLK_NB "s_cmp_eq_u32 %1, 0\n v_add_f32 %0, 1.0, %0\n"

template <int MODE>
__global__ void __launch_bounds__(256) kbr(int k, int iters, float* out) {
  float acc = threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) {
    if (MODE == 2) {
      asm volatile(BLK_NB BLK_NB BLK_NB BLK_NB BLK_NB BLK_NB BLK_NB BLK_NB : "+v"(acc) : "s"(k) : "scc");
    } else {
      asm volatile(BLK_BR BLK_BR BLK_BR BLK_BR BLK_BR BLK_BR BLK_BR BLK_BR : "+v"(acc) : "s"(k) : "scc");
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE>
float run(int k, int blocks, int iters, float* d) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  kbr<MODE><<<blocks, 256>>>(k, 100, d);
  (void)hipEventRecord(a);
  kbr<MODE><<<blocks, 256>>>(k, iters, d);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  float* d;
  (void)hipMalloc(&d, 1 << 24);
  const int iters = 200000;
  for (int w : {1, 4}) {
    const int blocks = 256 * w;
    float t0 = run<0>(0, blocks, iters, d);
    float t1 = run<0>(1, blocks, iters, d);
    float t2 = run<2>(0, blocks, iters, d);
    printf("waves/SIMD=%d  per block-of-8 per wave: taken %.2f ns, not-taken+valu %.2f ns, no-branch+valu %.2f ns\n",
           w, t0 * 1e6 / iters / 8 / w, t1 * 1e6 / iters / 8 / w, t2 * 1e6 / iters / 8 / w);
  }
  return 0;
}

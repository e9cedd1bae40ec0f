// Microbenchmark: issue cost of SALU / VALU / branch instruction streams on gfx950 as a
// function of waves per SIMD.  Prints cycles per instruction per wave and per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define SALU8 "s_add_u32 s20, s20, 1\n s_add_u32 s21, s21, 1\n s_add_u32 s22, s22, 1\n s_add_u32 s23, s23, 1\n" \
              "s_add_u32 s24, s24, 1\n s_add_u32 s25, s25, 1\n s_add_u32 s26, s26, 1\n s_add_u32 s27, s27, 1\n"
#define VALU8 "v_add_f32 v20, 1.0, v20\n v_add_f32 v21, 1.0, v21\n v_add_f32 v22, 1.0, v22\n v_add_f32 v23, 1.0, v23\n" \
              "v_add_f32 v24, 1.0, v24\n v_add_f32 v25, 1.0, v25\n v_add_f32 v26, 1.0, v26\n v_add_f32 v27, 1.0, v27\n"
#define MIX8 "s_add_u32 s20, s20, 1\n v_add_f32 v20, 1.0, v20\n s_add_u32 s21, s21, 1\n v_add_f32 v21, 1.0, v21\n" \
             "s_add_u32 s22, s22, 1\n v_add_f32 v22, 1.0, v22\n s_add_u32 s23, s23, 1\n v_add_f32 v23, 1.0, v23\n"
#define BR8 "s_cmp_eq_u32 s20, 12345\n s_cbranch_scc1 1f\n 1:\n s_cmp_eq_u32 s21, 12345\n s_cbranch_scc1 1f\n 1:\n" \
            "s_cmp_eq_u32 s22, 12345\n s_cbranch_scc1 1f\n 1:\n s_cmp_eq_u32 s23, 12345\n s_cbranch_scc1 1f\n 1:\n"
#define TBR8 "s_branch 1f\n 1:\n s_branch 1f\n 1:\n s_branch 1f\n 1:\n s_branch 1f\n 1:\n" \
             "s_branch 1f\n 1:\n s_branch 1f\n 1:\n s_branch 1f\n 1:\n s_branch 1f\n 1:\n"
#define CLOB "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "scc"

template <int MODE>
__global__ void k(long long* cyc, int iters) {
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) asm volatile(R8(SALU8) ::: CLOB);   // 64 SALU
    if (MODE == 1) asm volatile(R8(VALU8) ::: CLOB);   // 64 VALU
    if (MODE == 2) asm volatile(R8(MIX8) ::: CLOB);    // 32 SALU + 32 VALU
    if (MODE == 3) asm volatile(R8(BR8) ::: CLOB);     // 32 SALU + 32 not-taken cbranch
    if (MODE == 4) asm volatile(R8(TBR8) ::: CLOB);    // 64 taken s_branch
  }
  long long t1 = clock64();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  long long* cyc;
  (void)hipMalloc(&cyc, 1 << 20);
  const int iters = 2000;
  const char* names[] = {"64 SALU", "64 VALU", "32 SALU+32 VALU", "32 SALU+32 cbranch(not taken)", "64 s_branch(taken)"};
  for (int mode = 0; mode < 5; ++mode) {
    for (int threads : {64, 256, 512, 1024}) {
      auto kern = mode == 0 ? k<0> : mode == 1 ? k<1> : mode == 2 ? k<2> : mode == 3 ? k<3> : k<4>;
      // 256 blocks -> one block per CU (roughly); waves per SIMD = threads/256
      hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, cyc, iters);
      (void)hipDeviceSynchronize();
      long long c[16];
      (void)hipMemcpy(c, cyc, sizeof c, hipMemcpyDeviceToHost);
      double mx = 0;
      for (int w = 0; w < threads / 64; ++w) mx = c[w] > mx ? c[w] : mx;
      const double per_inst = mx / iters / 64.0;
      printf("%-32s waves/CU %2d: %.2f cyc/instr per wave, %.2f cyc/instr per SIMD\n", names[mode], threads / 64,
             per_inst, per_inst / ((threads / 64 + 3) / 4));
    }
  }
  return 0;
}

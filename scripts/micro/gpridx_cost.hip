// Microbenchmark: cost of a uniform-indexed VGPR read (s_set_gpr_idx / v_movrels) vs an LDS
// read vs a static register read, inside a dependent chain.  Prints cycles per iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef float f16v __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ void k(const int* idx, float* out, long long* cyc, int iters) {
  __shared__ float lds[16 * 256];
  const int t = threadIdx.x;
  f16v v;
  for (int i = 0; i < 16; ++i) { v[i] = (float)(i + t); lds[i * 256 + t] = (float)(i + t); }
  __syncthreads();
  float acc = 0.f;
  long long t0 = clock64();
#pragma unroll 8
  for (int it = 0; it < iters; ++it) {
    const int j = __builtin_amdgcn_readfirstlane((it * 7 + (int)idx[0]) & 15);
    float x;
    if (MODE == 0) x = v[j];                 // gpr_idx
    else if (MODE == 1) x = lds[j * 256 + t];  // LDS
    else x = v[(it & 7) + 4];                 // static index (loop unrolled)
    acc = __builtin_fmaf(acc, 0.999f, x);
    if (MODE == 0) v[(j + 1) & 15] = acc;    // gpr_idx write
    else if (MODE == 1) lds[((j + 1) & 15) * 256 + t] = acc;
  }
  long long t1 = clock64();
  out[blockIdx.x * blockDim.x + t] = acc;
  if (t == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  int* idx; float* out; long long* cyc;
  hipMalloc(&idx, 64 * 4); hipMalloc(&out, 1 << 24); hipMalloc(&cyc, 1 << 20);
  int h[64]; for (int i = 0; i < 64; ++i) h[i] = (i * 7) & 15;
  hipMemcpy(idx, h, sizeof h, hipMemcpyHostToDevice);
  const int iters = 4096;
  for (int blocks : {1, 1024}) {
    for (int threads : {64, 256}) {
      for (int mode = 0; mode < 3; ++mode) {
        auto kern = mode == 0 ? k<0> : (mode == 1 ? k<1> : k<2>);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, idx, out, cyc, iters);
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipEventRecord(a);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, idx, out, cyc, iters);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("mode %d (%s) blocks %d threads %d: %.1f cyc/iter (wave0), kernel %.3f ms\n", mode,
               mode == 0 ? "gpr_idx" : (mode == 1 ? "lds" : "static"), blocks, threads, (double)c / iters, ms);
      }
    }
  }
  return 0;
}

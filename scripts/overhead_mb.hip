// Microbenchmark for the per-step schedule / JIT-layout kernels (DESIGN.md "Round 6",
// per-step overhead): the one-block size scan and the one-block counting-sort schedule, each in
// the shipped form and a candidate form, on C3-shaped inputs.  Standalone (hipcc, no library):
//   hipcc --offload-arch=gfx950 -O3 scripts/overhead_mb.hip -o /tmp/overhead_mb && /tmp/overhead_mb
// Prints the average duration per launch (HIP events over 400 launches) and checks that the
// candidate forms agree with the shipped ones.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

constexpr int kWave = 64;
constexpr uint64_t kTmpl = 1024;  // stands in for mtgp::kJitTemplateBytes
constexpr int kBins = 4096;       // MTGP_SCHED_BINS

// ---- size scan: shipped form (each thread loads its PER contiguous sizes from global memory)
template <int PER>
__global__ void __launch_bounds__(1024) scan_reg(const uint32_t* __restrict__ src, uint32_t* __restrict__ offs,
                                                 int total, int32_t* __restrict__ info) {
  __shared__ uint64_t wsum[16];
  __shared__ int32_t werr[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int b = t * PER;
  uint32_t v[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) v[k] = (b + k < total) ? src[b + k] : 0u;
  uint64_t sum = 0;
  int bad = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const bool isbad = (v[k] & 0x80000000u) != 0u;
    const int code = -(int)(v[k] & 0x7fffffffu);
    bad = (isbad && code < bad) ? code : bad;
    sum += isbad ? 0u : v[k];
  }
  uint64_t inc = sum;
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t y = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += y;
  }
  int e = bad;
  for (int d = 1; d < kWave; d <<= 1) {
    const int o = __shfl_xor(e, d, kWave);
    e = o < e ? o : e;
  }
  if (lane == kWave - 1) wsum[w] = inc;
  if (lane == 0) werr[w] = e;
  __syncthreads();
  uint64_t wbase = 0;
  int err = 0;
  for (int q = 0; q < 16; ++q) {
    if (q < w) wbase += wsum[q];
    err = werr[q] < err ? werr[q] : err;
  }
  uint64_t run = wbase + inc - sum + kTmpl;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (b + k < total) {
      offs[b + k] = (uint32_t)(run < 0xffffffffull ? run : 0xffffffffull);
      run += (v[k] & 0x80000000u) ? 0u : v[k];
    }
  }
  if (t == 1023) {
    const uint64_t tot = wbase + inc + kTmpl;
    offs[total] = (uint32_t)(tot < 0xffffffffull ? tot : 0xffffffffull);
    info[0] = err;
    info[1] = (int32_t)(tot < 0x7fffffffull ? tot : 0x7fffffffull);
  }
}

// ---- size scan, candidate: coalesced global loads / stores, transposed through LDS (one word of
// padding per 64 so the per-thread contiguous reads are conflict-free on 64 banks)
__device__ __forceinline__ int lds_ix(int i) { return i + (i >> 6); }
template <int PER>
__global__ void __launch_bounds__(1024) scan_lds(const uint32_t* __restrict__ src, uint32_t* __restrict__ offs,
                                                 int total, int32_t* __restrict__ info) {
  constexpr int N = 1024 * PER;
  __shared__ uint32_t s[N + N / 64];
  __shared__ uint64_t wsum[16];
  __shared__ int32_t werr[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  uint32_t v[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = k * 1024 + t;
    v[k] = i < total ? src[i] : 0u;
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) s[lds_ix(k * 1024 + t)] = v[k];
  __syncthreads();
  const int b = t * PER;
#pragma unroll
  for (int k = 0; k < PER; ++k) v[k] = s[lds_ix(b + k)];
  uint64_t sum = 0;
  int bad = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const bool isbad = (v[k] & 0x80000000u) != 0u;
    const int code = -(int)(v[k] & 0x7fffffffu);
    bad = (isbad && code < bad) ? code : bad;
    sum += isbad ? 0u : v[k];
  }
  uint64_t inc = sum;
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t y = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += y;
  }
  int e = bad;
  for (int d = 1; d < kWave; d <<= 1) {
    const int o = __shfl_xor(e, d, kWave);
    e = o < e ? o : e;
  }
  if (lane == kWave - 1) wsum[w] = inc;
  if (lane == 0) werr[w] = e;
  __syncthreads();
  uint64_t wbase = 0;
  int err = 0;
  for (int q = 0; q < 16; ++q) {
    if (q < w) wbase += wsum[q];
    err = werr[q] < err ? werr[q] : err;
  }
  uint64_t run = wbase + inc - sum + kTmpl;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    s[lds_ix(b + k)] = (uint32_t)(run < 0xffffffffull ? run : 0xffffffffull);
    run += (v[k] & 0x80000000u) ? 0u : v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int i = k * 1024 + t;
    if (i < total) offs[i] = s[lds_ix(i)];
  }
  if (t == 1023) {
    const uint64_t tot = wbase + inc + kTmpl;
    offs[total] = (uint32_t)(tot < 0xffffffffull ? tot : 0xffffffffull);
    info[0] = err;
    info[1] = (int32_t)(tot < 0x7fffffffull ? tot : 0x7fffffffull);
  }
}

// ---- schedule
struct SchedW {
  int32_t w[8];
};
__device__ __forceinline__ int sched_cost(const int32_t* plen, int p, int n_prog, const SchedW& W) {
  int c = 0;
  for (int j = 0; j < n_prog; ++j) c += W.w[j] * plen[(size_t)p * n_prog + j];
  return c < 0 ? 0 : (c >= kBins ? kBins - 1 : c);
}
__device__ __forceinline__ int sched_slot(int sr, int P, int G) {
  const int h = P / 2;
  if (G == 1) return P - 1 - sr;
  if (sr < h) return 2 * sr + 1;
  if (sr >= P - h) return 2 * (P - 1 - sr);
  return P - 1;
}

// shipped form: Hillis-Steele scan of the per-thread bin sums
__global__ void __launch_bounds__(1024) sched_fused(const int32_t* __restrict__ plen, int P, int n_prog, SchedW W,
                                                    int G, int32_t* __restrict__ order) {
  __shared__ int32_t hist[kBins];
  __shared__ int32_t part[1024];
  constexpr int kPer = kBins / 1024;
  const int t = threadIdx.x;
  for (int i = t; i < kBins; i += 1024) hist[i] = 0;
  __syncthreads();
  for (int p = t; p < P; p += 1024) atomicAdd(&hist[sched_cost(plen, p, n_prog, W)], 1);
  __syncthreads();
  int loc[kPer], sum = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) { loc[i] = sum; sum += hist[t * kPer + i]; }
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const int v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const int base = part[t] - sum;
#pragma unroll
  for (int i = 0; i < kPer; ++i) hist[t * kPer + i] = base + loc[i];
  __syncthreads();
  for (int p = t; p < P; p += 1024) order[sched_slot(atomicAdd(&hist[sched_cost(plen, p, n_prog, W)], 1), P, G)] = p;
}

// candidate: the costs computed once into registers (loads issued together), wave-shuffle scan
// plus the 16 wave totals (two barriers instead of twenty)
template <int KP>
__global__ void __launch_bounds__(1024) sched_fused2(const int32_t* __restrict__ plen, int P, int n_prog, SchedW W,
                                                     int G, int32_t* __restrict__ order) {
  __shared__ int32_t hist[kBins];
  __shared__ int32_t wsum[16];
  constexpr int kPer = kBins / 1024;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
#pragma unroll
  for (int i = 0; i < kPer; ++i) hist[i * 1024 + t] = 0;
  int c[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int p = k * 1024 + t;
    c[k] = p < P ? sched_cost(plen, p, n_prog, W) : -1;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KP; ++k)
    if (c[k] >= 0) atomicAdd(&hist[c[k]], 1);
  __syncthreads();
  int loc[kPer], sum = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) { loc[i] = sum; sum += hist[t * kPer + i]; }
  int inc = sum;
  for (int d = 1; d < kWave; d <<= 1) {
    const int y = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += y;
  }
  if (lane == kWave - 1) wsum[w] = inc;
  __syncthreads();
  int base = inc - sum;
  for (int q = 0; q < 16; ++q)
    if (q < w) base += wsum[q];
#pragma unroll
  for (int i = 0; i < kPer; ++i) hist[t * kPer + i] = base + loc[i];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KP; ++k)
    if (c[k] >= 0) order[sched_slot(atomicAdd(&hist[c[k]], 1), P, G)] = k * 1024 + t;
}


// candidate 3: as candidate 2, with the atomics aggregated over the lanes of a wave that share a
// bin (peer mask from 13 ballots over the key bits; one atomic per distinct bin per wave)
__device__ __forceinline__ uint64_t peer_mask(int key) {
  uint64_t m = ~0ull;
#pragma unroll
  for (int b = 0; b < 13; ++b) {
    const bool bit = (key >> b) & 1;
    const uint64_t bb = __ballot(bit);
    m &= bit ? bb : ~bb;
  }
  return m;
}
template <int KP>
__global__ void __launch_bounds__(1024) sched_fused3(const int32_t* __restrict__ plen, int P, int n_prog, SchedW W,
                                                     int G, int32_t* __restrict__ order) {
  __shared__ int32_t hist[kBins];
  __shared__ int32_t wsum[16];
  constexpr int kPer = kBins / 1024;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
  for (int i = 0; i < kPer; ++i) hist[i * 1024 + t] = 0;
  int c[KP];
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const int p = k * 1024 + t;
    c[k] = p < P ? sched_cost(plen, p, n_prog, W) : kBins;  // kBins: no individual
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const uint64_t m = peer_mask(c[k]);
    if (c[k] < kBins && (m & below) == 0ull) atomicAdd(&hist[c[k]], __popcll(m));
  }
  __syncthreads();
  int loc[kPer], sum = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) { loc[i] = sum; sum += hist[t * kPer + i]; }
  int inc = sum;
  for (int d = 1; d < kWave; d <<= 1) {
    const int y = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += y;
  }
  if (lane == kWave - 1) wsum[w] = inc;
  __syncthreads();
  int base = inc - sum;
  for (int q = 0; q < 16; ++q)
    if (q < w) base += wsum[q];
#pragma unroll
  for (int i = 0; i < kPer; ++i) hist[t * kPer + i] = base + loc[i];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < KP; ++k) {
    const uint64_t m = peer_mask(c[k]);
    const bool lead = (m & below) == 0ull;
    int s0 = 0;
    if (c[k] < kBins && lead) s0 = atomicAdd(&hist[c[k]], __popcll(m));
    s0 = __shfl(s0, __ffsll((unsigned long long)m) - 1, kWave);
    if (c[k] < kBins) order[sched_slot(s0 + __popcll(m & below), P, G)] = k * 1024 + t;
  }
}

template <class F>
static float time_us(F launch, int iters) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  launch();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(a, 0);
  for (int i = 0; i < iters; ++i) launch();
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return ms * 1000.f / iters;
}

int main() {
  std::mt19937 rng(7);
  int fails = 0;
  // ---- scans: C3 n_units = 16384 (PER 16); 32768 (PER 32); a ragged total; error entries
  for (int total : {16384, 12345, 32768}) {
    for (int with_err : {0, 1}) {
      std::vector<uint32_t> h(total);
      for (auto& x : h) x = 64u * (3u + rng() % 40u);
      if (with_err) {
        h[total / 3] = 0x80000000u | 5u;
        h[total - 1] = 0x80000000u | 9u;
      }
      uint32_t *src, *o1, *o2;
      int32_t *i1, *i2;
      CK(hipMalloc(&src, total * 4));
      CK(hipMalloc(&o1, (total + 1) * 4));
      CK(hipMalloc(&o2, (total + 1) * 4));
      CK(hipMalloc(&i1, 8));
      CK(hipMalloc(&i2, 8));
      CK(hipMemcpy(src, h.data(), total * 4, hipMemcpyHostToDevice));
      float ta, tb;
      if (total <= 16384) {
        ta = time_us([&] { hipLaunchKernelGGL(scan_reg<16>, dim3(1), dim3(1024), 0, 0, src, o1, total, i1); }, 400);
        tb = time_us([&] { hipLaunchKernelGGL(scan_lds<16>, dim3(1), dim3(1024), 0, 0, src, o2, total, i2); }, 400);
      } else {
        ta = time_us([&] { hipLaunchKernelGGL(scan_reg<32>, dim3(1), dim3(1024), 0, 0, src, o1, total, i1); }, 400);
        tb = time_us([&] { hipLaunchKernelGGL(scan_lds<32>, dim3(1), dim3(1024), 0, 0, src, o2, total, i2); }, 400);
      }
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      std::vector<uint32_t> r1(total + 1), r2(total + 1);
      int32_t f1[2], f2[2];
      CK(hipMemcpy(r1.data(), o1, (total + 1) * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r2.data(), o2, (total + 1) * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(f1, i1, 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(f2, i2, 8, hipMemcpyDeviceToHost));
      // host expectation
      uint64_t run = kTmpl;
      int err = 0;
      bool ok = true;
      for (int i = 0; i < total; ++i) {
        if (r1[i] != (uint32_t)run || r2[i] != (uint32_t)run) ok = false;
        if (h[i] & 0x80000000u) err = std::min(err, -(int)(h[i] & 0x7fffffffu));
        else run += h[i];
      }
      ok = ok && r1[total] == (uint32_t)run && r2[total] == (uint32_t)run && f1[0] == err && f2[0] == err &&
           f1[1] == (int32_t)run && f2[1] == (int32_t)run;
      std::printf("scan total=%d err=%d  shipped %.2f us  lds %.2f us  %s\n", total, with_err, ta, tb,
                  ok ? "ok" : "MISMATCH");
      fails += !ok;
      CK(hipFree(src));
      CK(hipFree(o1));
      CK(hipFree(o2));
      CK(hipFree(i1));
      CK(hipFree(i2));
    }
  }
  // ---- schedule: C3 P = 8192 individuals x 2 programs; a ragged P; G = 1 and G = 2
  for (int narrow : {0, 1})
  for (int P : {8192, 5001}) {
    for (int G : {2, 1}) {
      const int n_prog = 2;
      std::vector<int32_t> pl((size_t)P * n_prog);
      for (auto& x : pl) x = narrow ? 20 + (int)(rng() % 6u) : 3 + (int)(rng() % 60u);
      SchedW W{};
      W.w[0] = 1;
      W.w[1] = 2;
      int32_t *plen, *o1, *o2;
      CK(hipMalloc(&plen, pl.size() * 4));
      CK(hipMalloc(&o1, P * 4));
      CK(hipMalloc(&o2, P * 4));
      CK(hipMemcpy(plen, pl.data(), pl.size() * 4, hipMemcpyHostToDevice));
      const float ta =
          time_us([&] { hipLaunchKernelGGL(sched_fused, dim3(1), dim3(1024), 0, 0, plen, P, n_prog, W, G, o1); }, 400);
      const float tb = time_us(
          [&] { hipLaunchKernelGGL(sched_fused2<8>, dim3(1), dim3(1024), 0, 0, plen, P, n_prog, W, G, o2); }, 400);
      int32_t* o3;
      CK(hipMalloc(&o3, P * 4));
      const float tc = time_us(
          [&] { hipLaunchKernelGGL(sched_fused3<8>, dim3(1), dim3(1024), 0, 0, plen, P, n_prog, W, G, o3); }, 400);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      std::vector<int32_t> r1(P), r2(P), r3(P);
      CK(hipMemcpy(r3.data(), o3, P * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r1.data(), o1, P * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r2.data(), o2, P * 4, hipMemcpyDeviceToHost));
      // both permutations, and the same cost in every slot (ties are ordered arbitrarily)
      auto cost = [&](int p) { return std::min(kBins - 1, pl[(size_t)p * 2] + 2 * pl[(size_t)p * 2 + 1]); };
      std::vector<int32_t> s1 = r1, s2 = r2, s3 = r3;
      std::sort(s1.begin(), s1.end());
      std::sort(s2.begin(), s2.end());
      std::sort(s3.begin(), s3.end());
      bool ok = true;
      for (int q = 0; q < P; ++q)
        ok = ok && s1[q] == q && s2[q] == q && s3[q] == q && cost(r1[q]) == cost(r2[q]) && cost(r1[q]) == cost(r3[q]);
      std::printf("sched %s P=%d G=%d  shipped %.2f us  fused2 %.2f us  fused3 %.2f us  %s\n",
                  narrow ? "narrow" : "wide", P, G, ta, tb, tc, ok ? "ok" : "MISMATCH");
      CK(hipFree(o3));
      fails += !ok;
      CK(hipFree(plen));
      CK(hipFree(o1));
      CK(hipFree(o2));
    }
  }
  std::printf("%s\n", fails ? "FAILED" : "all ok");
  return fails ? 1 : 0;
}

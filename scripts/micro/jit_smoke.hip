// JIT smoke test: translate a few programs on the host, place the code in executable device
// memory (hsa_amd_memory_pool_allocate + HSA_AMD_MEMORY_POOL_EXECUTABLE_FLAG), call it from a
// kernel with s_swappc_b64 under the mtgp_jit.h register ABI and compare with host results.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <math.h>
#include <stdio.h>
#include <string.h>
#include <vector>
#include "mtgp.h"
#include "mtgp_f32math.h"
#include "../../multitreegp_amd/csrc/mtgp_jit.h"

static hsa_agent_t g_agent;
static hsa_amd_memory_pool_t g_pool;
static hsa_status_t find_gpu(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) { g_agent = a; return HSA_STATUS_INFO_BREAK; }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_pool(hsa_amd_memory_pool_t p, void*) {
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t fl = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
  if (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) { g_pool = p; return HSA_STATUS_INFO_BREAK; }
  return HSA_STATUS_SUCCESS;
}

__device__ __forceinline__ float jit_call(uint64_t addr, const float d[8], uint64_t& flag) {
  float acc;
  asm volatile("s_swappc_b64 s[30:31], %[tgt]"
               : "={v8}"(acc), "+{s[32:33]}"(flag)
               : [tgt] "s"(addr), "{v0}"(d[0]), "{v1}"(d[1]), "{v2}"(d[2]), "{v3}"(d[3]), "{v4}"(d[4]),
                 "{v5}"(d[5]), "{v6}"(d[6]), "{v7}"(d[7])
               : "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21",
                 "v22", "v23", "v24", "v25", "s30", "s31", "s34", "s35", "s36", "s37", "s38", "s39", "s40", "s41",
                 "s42", "s43", "s44", "s45", "vcc", "memory");
  return acc;
}

__global__ void k_copy(const uint32_t* src, uint32_t* dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

__global__ void k_run(uint64_t base, const uint32_t* offs, int nprog, const float* in, float* out, uint32_t* flags) {
  asm volatile("s_icache_inv");
  float d[8];
  for (int i = 0; i < 8; ++i) d[i] = in[i * 64 + threadIdx.x];
  for (int p = 0; p < nprog; ++p) {
    uint64_t fl = 0;
    const float r = jit_call(base + __builtin_amdgcn_readfirstlane(offs[p]), d, fl);
    out[p * 64 + threadIdx.x] = r;
    if (threadIdx.x == 0) flags[p] = (uint32_t)(fl != 0);
  }
}

// sweep: sin and cos JIT programs over many arguments (all magnitudes incl. the double path)
__global__ void k_sweep(uint64_t base, uint32_t off_sin, uint32_t off_cos, const float* xs, int n, float* os, float* oc,
                        uint32_t* flags) {
  asm volatile("s_icache_inv");
  for (int i0 = 0; i0 < n; i0 += 64) {
    float d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int i = i0 + (int)threadIdx.x;
    d[2] = i < n ? xs[i] : 0.0f;
    uint64_t fl = 0;
    const float s = jit_call(base + off_sin, d, fl);
    const float c = jit_call(base + off_cos, d, fl);
    if (i < n) { os[i] = s; oc[i] = c; }
    if (fl && threadIdx.x == 0) atomicAdd(flags, 1u);
  }
}

static MtgpInstr I(int op, uint32_t aux, float imm) { MtgpInstr x; x.op = (uint32_t)op << MTGP_OP_SHIFT | aux; x.imm = imm; return x; }
static MtgpInstr IS(int op, uint32_t aux, uint32_t slot) { MtgpInstr x; x.op = (uint32_t)op << MTGP_OP_SHIFT | aux; memcpy(&x.imm, &slot, 4); return x; }

int main() {
  if (hsa_init() != HSA_STATUS_SUCCESS) { printf("hsa_init failed\n"); return 1; }
  hsa_iterate_agents(find_gpu, nullptr);
  hsa_amd_agent_iterate_memory_pools(g_agent, find_pool, nullptr);
  const size_t bytes = 1 << 20;
  void* code = nullptr;
  hsa_status_t st = hsa_amd_memory_pool_allocate(g_pool, bytes, HSA_AMD_MEMORY_POOL_EXECUTABLE_FLAG, &code);
  printf("exec alloc status %d ptr %p\n", (int)st, code);
  if (st != HSA_STATUS_SUCCESS) return 2;
  const uint32_t SB = MTGP_SLOT_BYTES;
  std::vector<std::vector<MtgpInstr>> progs = {
      {I(MTGP_OP_LDC, 0, 2.5f), I(MTGP_OP_END, 0, 0)},                                      // 2.5
      {IS(MTGP_OP_LDV, 0, 1 * SB), I(MTGP_OP_ADDC, 0, 0.75f), I(MTGP_OP_END, 0, 0)},         // d1 + .75
      {IS(MTGP_OP_SINV, 0, 2 * SB), I(MTGP_OP_END, 0, 0)},                                   // sin d2
      {IS(MTGP_OP_COSV, 0, 3 * SB), I(MTGP_OP_MULC, 0, 3.0f), I(MTGP_OP_END, 0, 0)},         // cos(d3) * 3
      {IS(MTGP_OP_VV_DIV, 5 * SB, 4 * SB), IS(MTGP_OP_LDVP, 0, 0), I(MTGP_OP_RSUBS, 0, 0), I(MTGP_OP_END, 0, 0)},  // RSUBS: d4/d5 - d0
      {IS(MTGP_OP_COSV, 0, 2 * SB), I(MTGP_OP_END, 0, 0)},                                   // cos d2 (sweep)
  };
  // shared subroutines first (mtgp_jit.h layout), then the programs
  std::vector<uint32_t> words(mtgp_jit_sub_blob, mtgp_jit_sub_blob + MTGP_JIT_SUB_WORDS), offs;
  for (auto& p : progs) {
    const uint32_t base = (uint32_t)(words.size() * 4);
    offs.push_back(base);
    const int n = mtgp::jit_translate(p.data(), (int)p.size(), nullptr, base);
    if (n < 0) { printf("translate error %d\n", n); return 3; }
    words.resize(words.size() + n);
    mtgp::jit_translate(p.data(), (int)p.size(), words.data() + words.size() - n, base);
    while (words.size() % 16) words.push_back(0xbf800000u);  // s_nop 0 padding to 64 B
  }
  uint32_t *dw, *doffs, *dflags;
  float *din, *dout;
  hipMalloc(&dw, words.size() * 4);
  hipMalloc(&doffs, offs.size() * 4);
  hipMalloc(&dflags, 64 * 4);
  hipMalloc(&din, 8 * 64 * 4);
  hipMalloc(&dout, progs.size() * 64 * 4);
  hipMemcpy(dw, words.data(), words.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(doffs, offs.data(), offs.size() * 4, hipMemcpyHostToDevice);
  float hin[8 * 64];
  for (int i = 0; i < 8 * 64; ++i) hin[i] = 0.37f * (float)(i % 64) - 5.0f + (float)(i / 64);
  hin[2 * 64 + 7] = 3.0e5f;  // a double-path sin argument in lane 7 (2^17 <= |x| < 2^28)
  hipMemcpy(din, hin, sizeof(hin), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_copy, dim3((words.size() + 255) / 256), dim3(256), 0, 0, dw, (uint32_t*)code, (int)words.size());
  hipDeviceSynchronize();
  hipLaunchKernelGGL(k_run, dim3(1), dim3(64), 0, 0, (uint64_t)code, doffs, (int)progs.size(), din, dout, dflags);
  hipError_t e = hipDeviceSynchronize();
  printf("run: %s\n", hipGetErrorString(e));
  if (e != hipSuccess) return 4;
  std::vector<float> hout(progs.size() * 64);
  uint32_t hfl[64];
  hipMemcpy(hout.data(), dout, hout.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hfl, dflags, progs.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    float d[8];
    for (int i = 0; i < 8; ++i) d[i] = hin[i * 64 + l];
    const float want[5] = {2.5f, d[1] + 0.75f, mtgp_sinf(d[2]), mtgp_cosf(d[3]) * 3.0f, d[4] / d[5] - d[0]};
    for (int p = 0; p < 5; ++p) {
      uint32_t a, b;
      memcpy(&a, &hout[p * 64 + l], 4);
      memcpy(&b, &want[p], 4);
      if (a != b) { if (bad < 10) printf("mismatch prog %d lane %d: %g vs %g\n", p, l, hout[p * 64 + l], want[p]); ++bad; }
    }
  }
  printf("flags: %u %u %u %u %u (expect 0 0 0 0 0: 3e5 now takes the double path)\n", hfl[0], hfl[1], hfl[2], hfl[3], hfl[4]);
  // sweep
  {
    const int n = 1 << 20;
    std::vector<float> xs(n);
    uint32_t st = 12345u;
    for (int i = 0; i < n; ++i) {
      st = st * 1664525u + 1013904223u;
      const float u = (float)(st >> 8) / 16777216.0f;
      const int band = i % 10;
      const float mag = band == 0 ? 4.0f : band == 1 ? 2.0e5f : band == 2 ? 1.5e8f : band == 3 ? 1.0e7f
                      : band == 4 ? 131072.0f * (1.0f + u) : band == 5 ? 268435456.0f * 0.999f
                      : band == 6 ? 268435456.0f * (1.0f + 3.0f * u) : band == 7 ? 1.0e12f
                      : band == 8 ? 1.0e25f : 3.0e38f;
      xs[i] = (u * 2.0f - 1.0f) * mag;
    }
    xs[0] = 131072.0f; xs[1] = -131072.0f; xs[2] = 268435440.0f; xs[3] = 1e-30f; xs[4] = -0.0f;
    xs[5] = 268435456.0f; xs[6] = -268435456.0f; xs[7] = 3.4028235e38f; xs[8] = -3.4028235e38f;
    xs[9] = 1.0f / 0.0f; xs[10] = -1.0f / 0.0f; xs[11] = __builtin_nanf("");
    float *dx, *ds, *dc;
    uint32_t* dfl;
    hipMalloc(&dx, n * 4); hipMalloc(&ds, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&dfl, 4);
    hipMemcpy(dx, xs.data(), n * 4, hipMemcpyHostToDevice);
    hipMemset(dfl, 0, 4);
    hipLaunchKernelGGL(k_sweep, dim3(1), dim3(64), 0, 0, (uint64_t)code, offs[2], offs[5], dx, n, ds, dc, dfl);
    hipError_t e2 = hipDeviceSynchronize();
    printf("sweep: %s\n", hipGetErrorString(e2));
    std::vector<float> hs(n), hc(n);
    uint32_t nfl = 0;
    hipMemcpy(hs.data(), ds, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(hc.data(), dc, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(&nfl, dfl, 4, hipMemcpyDeviceToHost);
    int sb = 0;
    for (int i = 0; i < n; ++i) {
      const float ws = mtgp_sinf(xs[i]), wc = mtgp_cosf(xs[i]);
      uint32_t a, b, c2, d2;
      memcpy(&a, &hs[i], 4); memcpy(&b, &ws, 4); memcpy(&c2, &hc[i], 4); memcpy(&d2, &wc, 4);
      const bool nan_ok = (hs[i] != hs[i] && ws != ws) && (hc[i] != hc[i] && wc != wc);
      if ((a != b || c2 != d2) && !nan_ok) { if (sb < 5) printf("sweep mismatch x=%.9g sin %.9g/%.9g cos %.9g/%.9g\n", xs[i], hs[i], ws, hc[i], wc); ++sb; }
    }
    printf("sweep: %d mismatches of %d, fallback flags %u (expect 0)\n", sb, n, nfl);
    bad += sb + (int)nfl;
  }
  printf("%s: %d mismatches\n", bad ? "FAIL" : "OK", bad);
  hsa_amd_memory_pool_free(code);
  return bad ? 5 : 0;
}

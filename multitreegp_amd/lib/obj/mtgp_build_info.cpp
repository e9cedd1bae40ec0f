#include <cstdint>
#include <cstring>
static const char kInfo[] = "sources_sha256=b0e7f1bd248c31e554fa703447862c0f413018817a2c8b12dbbe275f4b9a3f73;abi_header=include/mtgp.h";
extern "C" int mtgp_build_info(char* out, int32_t cap) {
  const int n = (int)sizeof(kInfo) - 1;
  if (out && cap > 0) { const int m = n < cap - 1 ? n : cap - 1; std::memcpy(out, kInfo, m); out[m] = 0; }
  return n;
}

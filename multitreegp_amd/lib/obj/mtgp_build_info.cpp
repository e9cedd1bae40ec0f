#include <cstdint>
#include <cstring>
static const char kInfo[] = "sources_sha256=5928e9f8ab956a9c4372edafea1c39101f7428c05226b33794b8cb9fd1edb2de;abi_header=include/mtgp.h";
extern "C" int mtgp_build_info(char* out, int32_t cap) {
  const int n = (int)sizeof(kInfo) - 1;
  if (out && cap > 0) { const int m = n < cap - 1 ? n : cap - 1; std::memcpy(out, kInfo, m); out[m] = 0; }
  return n;
}

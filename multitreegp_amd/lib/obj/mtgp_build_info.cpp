#include <cstdint>
#include <cstring>
static const char kInfo[] = "sources_sha256=e655132105b8c675aef5cdc35e71bbafde5af9268caf52f32d869c889ab2f95f;abi_header=include/mtgp.h";
extern "C" int mtgp_build_info(char* out, int32_t cap) {
  const int n = (int)sizeof(kInfo) - 1;
  if (out && cap > 0) { const int m = n < cap - 1 ? n : cap - 1; std::memcpy(out, kInfo, m); out[m] = 0; }
  return n;
}

// CRC32C (Castagnoli) for TF tensor-bundle checkpoints (manette_amd/tf_bundle.py): the SSE4.2
// crc32 instruction, 8 bytes per step. Declared in include/manette_host.h.
#include <nmmintrin.h>

#include <cstddef>
#include <cstdint>
#include <cstring>

#include "../../include/manette_host.h"

extern "C" uint32_t mh_crc32c(const void *data, size_t n, uint32_t crc) {
  const uint8_t *p = static_cast<const uint8_t *>(data);
  uint64_t c = ~crc & 0xffffffffu;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}

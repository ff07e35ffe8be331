// Block-key hashing shared by the engine KV manager (APC), the KV-event
// publisher and the router's precise prefix index, so the same token prefix
// produces the same chained 64-bit block keys everywhere.
//   key_i = H(key_{i-1}, extra_key, tokens of block i)
// (reference semantics: BlockStored carries the parent hash and the block's
// tokens, docs/architecture/advanced/kv-management/kv-indexer.md:57-87)
#pragma once
#include <cstddef>
#include <cstdint>

namespace llmd_rt {

inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

constexpr uint64_t kRootHash = 0x6c6c6d2d642d616dull;  // "llm-d-am"

inline uint64_t hash_block(uint64_t parent, uint64_t extra, const int32_t* toks, size_t n) {
  uint64_t h = mix64(parent ^ 0x9e3779b97f4a7c15ull) ^ mix64(extra + 0x632be59bd9b4e019ull);
  size_t i = 0;
  for (; i + 1 < n; i += 2) {
    const uint64_t w = (uint64_t)(uint32_t)toks[i] | ((uint64_t)(uint32_t)toks[i + 1] << 32);
    h = mix64(h ^ w) + 0x9e3779b97f4a7c15ull;
  }
  if (i < n) h = mix64(h ^ (uint64_t)(uint32_t)toks[i] ^ 0xff51afd7ed558ccdull);
  h = mix64(h ^ (uint64_t)n);
  return h == 0 ? 1 : h;  // 0 is reserved for "no hash"
}

}  // namespace llmd_rt

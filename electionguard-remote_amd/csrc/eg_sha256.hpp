// eg_sha256.hpp — device SHA-256 for the Fiat-Shamir challenges of the ballot
// proofs (one thread per hash, 64-byte block buffer in LDS).
//
// The pre-image is EG 1.0-style hash_elems: "|" + hex(e_0) + "|" + ... + "|", with
// ElementModP as 1024 and ElementModQ as 64 upper-case hex chars (fixed width,
// common.proto:6-16).  The upstream (electionguard-kotlin-multiplatform) format is
// not in the container: unpinned; this matches oracle/eg_oracle.py:hash_elems.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace eg {

__device__ __constant__ const uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

struct Sha256 {
  uint32_t* buf;  // 16 words of LDS owned by this thread (the current 64-byte block)
  uint32_t h[8];
  uint32_t len;   // bytes so far
  uint32_t pend;  // the block word being filled: bytes [len & ~3, len) in its low bytes

  __device__ __forceinline__ void init(uint32_t* lds_words) {
    buf = lds_words;
    h[0] = 0x6a09e667; h[1] = 0xbb67ae85; h[2] = 0x3c6ef372; h[3] = 0xa54ff53a;
    h[4] = 0x510e527f; h[5] = 0x9b05688c; h[6] = 0x1f83d9ab; h[7] = 0x5be0cd19;
    len = 0;
    pend = 0;
  }

  __device__ void compress() {
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) w[t] = __builtin_bswap32(buf[t]);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int t = 0; t < 64; ++t) {
      uint32_t wt;
      if (t < 16) {
        wt = w[t];
      } else {
        const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
        const uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
        const uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
        wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
        w[t & 15] = wt;
      }
      const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = hh + S1 + ch + kSha256K[t] + wt;
      const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
      const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      const uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }

  // one byte
  __device__ __forceinline__ void put(uint32_t ch) {
    pend |= (ch & 0xFFu) << (8 * (len & 3));
    ++len;
    if ((len & 3) == 0) {
      buf[((len >> 2) - 1) & 15] = pend;
      pend = 0;
      if ((len & 63) == 0) compress();
    }
  }

  // four bytes at once (v's low byte first): one LDS word store instead of four byte stores;
  // at a byte offset k = len & 3 the first 4 - k bytes complete the pending word
  __device__ __forceinline__ void put4(uint32_t v) {
    const uint32_t k = len & 3, wi = (len >> 2) & 15;
    if (k == 0) {
      buf[wi] = v;
    } else {
      buf[wi] = pend | (v << (8 * k));
      pend = v >> (32 - 8 * k);
    }
    len += 4;
    if (wi == 15) compress();
  }

  __device__ __forceinline__ static uint32_t hexc(uint32_t v) { return v < 10 ? ('0' + v) : ('A' + v - 10); }

  // four nibbles (one per byte, 0..15) -> four upper-case hex characters, bytewise SWAR
  __device__ __forceinline__ static uint32_t hex4(uint32_t n) {
    const uint32_t ge10 = ((n + 0x06060606u) >> 4) & 0x01010101u;  // nibble >= 10
    return n + 0x30303030u + (ge10 << 3) - ge10;                     // '0' + n (+ 7 for A-F)
  }

  // Upper-case hex of n big-endian bytes.  minimal = false: fixed width (2n chars, n a
  // multiple of 16, 16-B aligned source), 8 characters per source word through put4;
  // minimal = true: leading zero BYTES dropped, at least one kept (the integer's even-length
  // hex, e.g. 0 -> "00", 0xABC -> "0ABC": electionguard-python 1.x to_hex), a byte at a
  // time; see eg_ctx_set_hash_format.
  __device__ void put_hex(const uint8_t* __restrict__ p, uint32_t n, bool minimal = false) {
    const uint4* s = reinterpret_cast<const uint4*>(p);
    if (!minimal) {
      for (uint32_t i = 0; i < n / 16; ++i) {
        const uint4 v = s[i];
        const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t lo = ws[k] & 0x0F0F0F0Fu, hi = (ws[k] >> 4) & 0x0F0F0F0Fu;
          // bytes b0..b3 in memory order -> characters hi(b0) lo(b0) hi(b1) lo(b1) | hi(b2) ...
          put4(hex4(__builtin_amdgcn_perm(hi, lo, 0x01050004u)));
          put4(hex4(__builtin_amdgcn_perm(hi, lo, 0x03070206u)));
        }
      }
      return;
    }
    uint32_t first = 0;
    while (first + 1 < n && p[first] == 0) ++first;
    for (uint32_t i = first / 16; i < n / 16; ++i) {
      const uint4 v = s[i];
      const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint32_t idx = i * 16 + k * 4 + b;
          if (idx < first) continue;
          const uint32_t byte = (ws[k] >> (8 * b)) & 0xFF;
          put(hexc(byte >> 4));
          put(hexc(byte & 15));
        }
      }
    }
  }

  __device__ void finish(uint32_t (&dig)[8]) {
    const uint64_t bits = (uint64_t)len * 8;
    put(0x80);
    while ((len & 63) != 56) put(0);
    for (int i = 7; i >= 0; --i) put((uint32_t)(bits >> (8 * i)) & 0xFF);
#pragma unroll
    for (int i = 0; i < 8; ++i) dig[i] = h[i];
  }
};

}  // namespace eg

// hbx_deflate.hip — zlib block compression on gfx950.
//
// Reference: HashboxBlock.CompressData -> zlibCompress (pkg/core/block.go:
// 133-150, 176-184): Go compress/zlib at DefaultCompression over each block's
// data, done by the client's workers before a block is sent (pkg/core/
// client.go:249-258).  The output need not be bit-identical: the server
// inflates and re-hashes (block.go:159-166) and DataType is not hashed
// (block.go:101).  What must hold is that the stream is valid zlib (RFC 1950/
// 1951) and inflates to the block's data; that is what the tests check.
//
// Layout of one block's stream (all segments independent, so one workgroup
// per 32 KiB segment, no serial dependence between segments):
//
//   78 9C | seg 0 | seg 1 | ... | 01 00 00 FF FF | adler32 (BE)
//
//   seg = one non-final fixed-Huffman block (BTYPE 01) of LZ77 tokens whose
//         matches stay inside the segment, closed by an empty stored block
//         (a sync flush: 3 zero bits, pad, 00 00 FF FF) so the segment ends on
//         a byte boundary; or, if that is not smaller, one non-final stored
//         block (00 | LEN | ~LEN | data).
//
// K7a hbx_k7_deflate_size   per segment: LZ77 parse, coded image into a
//                           scratch slot, its size, mode and Adler partials
// K7s hbx_k7_deflate_plan   per block: segment offsets, header, trailer with
//                           the combined Adler-32, stream length
// K7b hbx_k7_deflate_write  per segment: its image from the slot to the
//                           stream at its byte offset
//
// The LZ77 parse (one 512-thread workgroup per 32 KiB segment, all in LDS):
//   1. candidates, in position order: round r covers positions 512r..512r+511
//      (thread t: 512r+t).  A 2048 x 4 hash table of 4-byte prefixes holds,
//      per hash and per position residue mod 4, the latest position inserted
//      so far (ds_max, no lock; one barrier per round, so a slot may already
//      hold a later position of the same round, which is skipped).  Each thread keeps the
//      longest verified match among its <= 4 candidates (as a distance).
//   2. thread t parses its own 64-byte range greedily with those distances,
//      one-step lazy (a longer match at p+1 defers p as a literal, as zlib's
//      lazy matching does), a match growing 4 bytes per compare up to 258 or
//      the range end; it counts the fixed-Huffman bits;
//   3. after a workgroup prefix sum of the bit counts, the same parse emits
//      the bits (ds_or) into the image, if that is smaller than stored.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hbxz {

constexpr uint32_t kSeg = 32768;  // bytes per segment (one workgroup)
constexpr uint32_t kThreads = 512;
constexpr uint32_t kWaves = kThreads / 64;
constexpr uint32_t kSub = kSeg / kThreads;  // 64 bytes per thread in the parse
constexpr uint32_t kHashBits = 11;
constexpr uint32_t kWays = 4;
constexpr uint32_t kDataWords = kSeg / 4 + 4;        // + slack for 4-byte reads past the end
// The segment and the candidate array live in LDS with one pad dword per
// parse range (kSub/4 data dwords, kSub/2 candidate dwords): thread t's range
// starts kSub bytes after thread t-1's, which without padding puts the 64
// lanes of a wave on a few banks.
constexpr uint32_t kDataShift = 31 - __builtin_clz(kSub / 4);
constexpr uint32_t kCdShift = 31 - __builtin_clz(kSub / 2);
constexpr uint32_t kDataPhys = kDataWords + (kDataWords >> kDataShift) + 1;
constexpr uint32_t kCdPhys = (kSeg / 2 + (kSeg / 2 >> kCdShift)) * 2;  // u16 slots
constexpr uint32_t kImgWords = (kSeg + 16) / 4 + 4;  // stored image (5 + kSeg) or a smaller fixed one
constexpr uint32_t kTabWords = (1u << kHashBits) * kWays;
constexpr uint32_t kSlot = kImgWords * 4;  // scratch bytes per segment
constexpr uint32_t kAdlerMod = 65521;
constexpr uint32_t kLazy = 32;  // no look-ahead past a match this long

struct SegInfo {
  uint32_t bytes;  // coded bytes of the segment (stored or fixed image)
  uint32_t mode;   // 0 stored, 1 fixed Huffman
  uint32_t a, b;   // Adler partials: sum x, sum (n - j) x_j  (mod 65521)
};

// Descriptor of one block to compress.
struct ZBlock {
  uint64_t src;   // device address of the data
  uint64_t dst;   // device address of the output stream
  uint64_t len;   // data bytes
  uint32_t seg0;  // first global segment index
  uint32_t nseg;  // ceil(len / kSeg)
};

__device__ __forceinline__ uint32_t lds4(const uint32_t* w, uint32_t p) {
  return __builtin_amdgcn_alignbyte(w[(p >> 2) + 1], w[p >> 2], p & 3u);
}
__device__ __forceinline__ uint32_t dphys(uint32_t k) { return k + (k >> kDataShift); }
// 4 bytes at byte p of the padded segment
__device__ __forceinline__ uint32_t seg4(const uint32_t* w, uint32_t p) {
  const uint32_t i = p >> 2;
  return __builtin_amdgcn_alignbyte(w[dphys(i + 1u)], w[dphys(i)], p & 3u);
}
__device__ __forceinline__ uint32_t cphys(uint32_t p) {
  const uint32_t wd = p >> 1;
  return 2u * (wd + (wd >> kCdShift)) + (p & 1u);
}

__device__ __forceinline__ uint32_t zhash(uint32_t x) { return (x * 0x9E3779B1u) >> (32 - kHashBits); }

// Fixed-code tables (RFC 1951 §3.2.5-3.2.6), as (reversed code | extra << n, n).
__device__ __forceinline__ uint32_t rev(uint32_t c, uint32_t n) { return __builtin_bitreverse32(c) >> (32u - n); }

__device__ __forceinline__ void lit_code(uint32_t x, uint32_t& v, uint32_t& n) {
  if (x < 144u) {
    n = 8u;
    v = rev(0x30u + x, 8u);
  } else {
    n = 9u;
    v = rev(0x190u + x - 144u, 9u);
  }
}

// match (len 4..258, dist 1..32768) -> one bit string of <= 31 bits
__device__ __forceinline__ void match_code(uint32_t len, uint32_t dist, uint32_t& v, uint32_t& n) {
  uint32_t sym, le = 0u, lx = 0u;
  if (len <= 10u) {
    sym = 254u + len;
  } else if (len == 258u) {
    sym = 285u;
  } else {
    const uint32_t l = len - 3u;
    le = 31u - __builtin_clz(l) - 2u;
    sym = 257u + 4u * (le + 1u) + ((l >> le) & 3u);
    lx = l & ((1u << le) - 1u);
  }
  uint32_t lv, ln;
  if (sym < 280u) {
    ln = 7u;
    lv = rev(sym - 256u, 7u);
  } else {
    ln = 8u;
    lv = rev(0xC0u + sym - 280u, 8u);
  }
  const uint32_t d = dist - 1u;
  uint32_t dc, de = 0u, dx = 0u;
  if (d < 4u) {
    dc = d;
  } else {
    de = 31u - __builtin_clz(d) - 1u;
    dc = 2u * (de + 1u) + ((d >> de) & 1u);
    dx = d & ((1u << de) - 1u);
  }
  v = lv | (lx << ln);
  n = ln + le;
  v |= (rev(dc, 5u) | (dx << 5)) << n;
  n += 5u + de;
}

// Segment bytes -> LDS words; word k holds data bytes [4k - sh, 4k - sh + 4)
// relative to the (4-byte aligned) base at src - sh.  Bytes past the segment
// come from the next bytes of the arena (always readable: HBX_ARENA_SLACK) and
// never take part in a match.
__device__ __forceinline__ void load_segment(uint32_t* data, const uint8_t* src, uint32_t n, uint32_t& sh) {
  const uint64_t a = reinterpret_cast<uint64_t>(src);
  sh = (uint32_t)(a & 3u);
  const uint32_t* base = reinterpret_cast<const uint32_t*>(a - sh);
  const uint32_t nw = (n + sh + 3u) >> 2;
  for (uint32_t k = threadIdx.x; k < kDataWords; k += kThreads) data[dphys(k)] = k < nw ? base[k] : 0u;
}

// Common prefix length of the strings at p and q (q < p), at most limit.
__device__ __forceinline__ uint32_t match_len(const uint32_t* data, uint32_t sh, uint32_t p, uint32_t q,
                                              uint32_t limit) {
  uint32_t len = 0u;
  while (len < limit) {
    const uint32_t dlt = seg4(data, p + len + sh) ^ seg4(data, q + len + sh);
    if (dlt) {
      len += (uint32_t)__builtin_ctz(dlt) >> 3;
      break;
    }
    len += 4u;
  }
  return min(len, limit);
}

// Steps 2/3: thread t's parse of [128t, 128t+128) ∩ [0, n) with the
// candidate distances `cd` (0 = none).  EMIT = false counts bits; EMIT = true
// ORs them into `img` from bit offset o.
template <bool EMIT>
__device__ __forceinline__ uint32_t parse_range(const uint32_t* data, const uint16_t* cd, uint32_t* img,
                                                uint32_t sh, uint32_t n, uint32_t o) {
  const uint32_t r0 = threadIdx.x * kSub;
  const uint32_t end = min(r0 + kSub, n);
  uint32_t bits = 0u, p = r0, len = 0u, d = 0u;
  bool have = false;  // (len, d) already hold the match at p
  while (p < end) {
    if (!have) {
      d = cd[cphys(p)];
      len = d ? match_len(data, sh, p, p - d, min(258u, end - p)) : 0u;
    }
    have = false;
    uint32_t v, nb, step;
    bool defer = false;
    if (len >= 4u && len < kLazy && p + 1u < end) {
      const uint32_t d1 = cd[cphys(p + 1u)];
      const uint32_t len1 = d1 ? match_len(data, sh, p + 1u, p + 1u - d1, min(258u, end - p - 1u)) : 0u;
      if (len1 > len) {  // lazy: p becomes a literal, the longer match starts at p + 1
        defer = true;
        len = len1;
        d = d1;
        have = true;
      }
    }
    if (len >= 4u && !defer) {
      match_code(len, d, v, nb);
      step = len;
    } else {
      lit_code(seg4(data, p + sh) & 0xFFu, v, nb);
      step = 1u;
    }
    if (EMIT) {
      const uint32_t w = o >> 5, s = o & 31u;
      atomicOr(&img[w], v << s);
      if (s + nb > 32u) atomicOr(&img[w + 1u], v >> (32u - s));
      o += nb;
    }
    bits += nb;
    p += step;
  }
  return bits;
}

// Inclusive prefix sum over the workgroup; `tot` = the total.
__device__ __forceinline__ uint32_t wg_incl_sum(uint32_t x, uint32_t* wsum, uint32_t& tot) {
  const uint32_t l = threadIdx.x & 63u, w = threadIdx.x >> 6;
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, d);
    if (l >= (uint32_t)d) x += y;
  }
  if (l == 63u) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0u;
  for (uint32_t k = 0; k < w; k++) before += wsum[k];
  tot = 0u;
  for (uint32_t k = 0; k < kWaves; k++) tot += wsum[k];
  __syncthreads();
  return before + x;
}

}  // namespace hbxz

// Global segment g -> its block (binary search over seg0).
__device__ __forceinline__ uint32_t zblock_of(const hbxz::ZBlock* blocks, uint32_t nb, uint32_t g) {
  uint32_t lo = 0, hi = nb - 1u;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1u) >> 1;
    if (blocks[mid].seg0 <= g)
      lo = mid;
    else
      hi = mid - 1u;
  }
  return lo;
}

extern "C" __global__ __launch_bounds__(512) void hbx_k7_deflate_size(const hbxz::ZBlock* __restrict__ blocks,
                                                                       uint32_t nb, uint32_t nseg,
                                                                       hbxz::SegInfo* __restrict__ info,
                                                                       uint32_t* __restrict__ scratch) {
  using namespace hbxz;
  __shared__ uint32_t data[kDataPhys];
  __shared__ uint32_t tab[kTabWords > kImgWords ? kTabWords : kImgWords];  // hash table, then the image
  __shared__ uint16_t cd[kCdPhys];
  __shared__ uint32_t wsum[kWaves];
  __shared__ unsigned long long wadler[2 * kWaves];
  const uint32_t g = blockIdx.x;
  if (g >= nseg) return;
  const ZBlock bk = blocks[zblock_of(blocks, nb, g)];
  const uint32_t s = g - bk.seg0;
  const uint64_t off = (uint64_t)s * kSeg;
  const uint32_t n = (uint32_t)min((uint64_t)kSeg, bk.len - off);
  const uint32_t t = threadIdx.x;
  uint32_t sh;
  load_segment(data, reinterpret_cast<const uint8_t*>(bk.src) + off, n, sh);
  for (uint32_t k = t; k < kTabWords; k += kThreads) tab[k] = 0u;
  __syncthreads();

  // 1. candidates in position order + Adler partials
  uint32_t A = 0u, J = 0u;  // sum x, sum j*x over this thread's positions (j < 32768: J < 2^32)
  for (uint32_t r = 0; r < kSeg / kThreads; r++) {
    const uint32_t p = kThreads * r + t;
    const uint32_t x = seg4(data, p + sh);
    const bool live = p + 4u <= n;
    const uint32_t h = zhash(x);
    uint32_t best = 0u, bl = 0u;
    if (live) {
      const uint4 c = *reinterpret_cast<const uint4*>(&tab[h * kWays]);
      const uint32_t lim = min(258u, n - p);
      const uint32_t cs[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int k = 0; k < 4; k++) {
        // a slot may already hold a later position of this round (no barrier
        // between reads and inserts): only earlier positions are candidates
        if (cs[k] != 0u && cs[k] - 1u < p && seg4(data, cs[k] - 1u + sh) == x) {
          const uint32_t q = cs[k] - 1u;
          const uint32_t L = 4u + match_len(data, sh, p + 4u, q + 4u, lim - 4u);
          if (L > bl || (L == bl && p - q < best)) {
            bl = L;
            best = p - q;
          }
        }
      }
    }
    cd[cphys(p)] = (uint16_t)best;
    if (p < n) {
      A += x & 0xFFu;
      J += p * (x & 0xFFu);
    }
    if (live) atomicMax(&tab[h * kWays + (p & (kWays - 1u))], p + 1u);
    __syncthreads();
  }

  // 2. count
  const uint32_t bits = parse_range<false>(data, cd, nullptr, sh, n, 0u);
  uint32_t tb;
  const uint32_t incl = wg_incl_sum(bits, wsum, tb);
  const uint32_t total_bits = 3u + tb + 7u + 3u;  // header, tokens, EOB, empty stored header
  const uint32_t fixed_bytes = ((total_bits + 7u) >> 3) + 4u;
  const uint32_t stored_bytes = 5u + n;
  const bool fixed = fixed_bytes < stored_bytes;
  uint32_t* img = tab;
  for (uint32_t k = t; k < kImgWords; k += kThreads) img[k] = 0u;
  __syncthreads();
  if (fixed) {
    // 3. emit: header bits 0..2 = BFINAL 0, BTYPE 01; EOB and the empty stored
    // block's header are zero bits; its LEN/NLEN on the next byte boundary
    if (t == 0) atomicOr(&img[0], 2u);
    parse_range<true>(data, cd, img, sh, n, 3u + incl - bits);
    __syncthreads();
    if (t == 0) {
      uint8_t* ob = reinterpret_cast<uint8_t*>(img);
      const uint32_t e = fixed_bytes - 4u;
      ob[e] = 0x00;
      ob[e + 1] = 0x00;
      ob[e + 2] = 0xFF;
      ob[e + 3] = 0xFF;
    }
  } else {
    // stored image: 00 | LEN | ~LEN | data
    for (uint32_t k = t; k < (n + 5u + 3u) / 4u; k += kThreads) {
      uint32_t w;
      if (k >= 2u) {
        w = seg4(data, 4u * k - 5u + sh);
      } else {
        const uint32_t d0 = seg4(data, sh);
        w = k == 0u ? ((n & 0xFFu) << 8) | (((n >> 8) & 0xFFu) << 16) | ((~n & 0xFFu) << 24)
                    : ((~n >> 8) & 0xFFu) | (d0 << 8);
      }
      img[k] = w;
    }
  }
  __syncthreads();
  const uint32_t nbytes = fixed ? fixed_bytes : stored_bytes;
  uint32_t* slot = scratch + (uint64_t)g * kImgWords;
  for (uint32_t k = t; k < (nbytes + 3u) / 4u; k += kThreads) slot[k] = img[k];

  // Adler partials: B = sum (n - j) x_j = n*A - J  (64-bit, then mod)
  unsigned long long A64 = A, J64 = J;
  for (int dd = 32; dd >= 1; dd >>= 1) {
    A64 += (unsigned long long)__shfl_xor((long long)A64, dd);
    J64 += (unsigned long long)__shfl_xor((long long)J64, dd);
  }
  if ((t & 63u) == 0u) {
    wadler[2 * (t >> 6)] = A64;
    wadler[2 * (t >> 6) + 1] = J64;
  }
  __syncthreads();
  if (t == 0) {
    unsigned long long As = 0, Js = 0;
    for (uint32_t k = 0; k < kWaves; k++) {
      As += wadler[2 * k];
      Js += wadler[2 * k + 1];
    }
    SegInfo si;
    si.mode = fixed ? 1u : 0u;
    si.bytes = nbytes;
    si.a = (uint32_t)(As % kAdlerMod);
    si.b = (uint32_t)(((unsigned long long)n * As - Js) % kAdlerMod);
    info[g] = si;
  }
}

// One wave per block: segment offsets (exclusive scan), header, trailer.
extern "C" __global__ __launch_bounds__(64) void hbx_k7_deflate_plan(const hbxz::ZBlock* __restrict__ blocks,
                                                                      uint32_t nb,
                                                                      const hbxz::SegInfo* __restrict__ info,
                                                                      uint64_t* __restrict__ seg_off,
                                                                      uint64_t* __restrict__ out_len) {
  using namespace hbxz;
  const uint32_t c = blockIdx.x;
  if (c >= nb) return;
  const ZBlock bk = blocks[c];
  const uint32_t l = threadIdx.x;
  uint64_t run = 2;  // after 78 9C
  uint32_t a = 1u, b = (uint32_t)(bk.len % kAdlerMod);
  for (uint32_t t = 0; t < bk.nseg; t += 64u) {
    const uint32_t s = t + l;
    uint32_t bytes = 0u, sa = 0u, sb = 0u;
    if (s < bk.nseg) {
      const SegInfo si = info[bk.seg0 + s];
      bytes = si.bytes;
      const uint64_t o = (uint64_t)s * kSeg;
      const uint64_t ns = min((uint64_t)kSeg, bk.len - o);
      const uint64_t after = bk.len - o - ns;  // bytes of the block after this segment
      sa = si.a;
      sb = (uint32_t)(((after % kAdlerMod) * si.a + si.b) % kAdlerMod);
    }
    uint32_t incl = bytes;
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, d);
      if (l >= (uint32_t)d) incl += y;
    }
    if (s < bk.nseg) seg_off[bk.seg0 + s] = bk.dst + run + (incl - bytes);
    for (int d = 32; d >= 1; d >>= 1) {
      sa += (uint32_t)__shfl_xor((int)sa, d);
      sb += (uint32_t)__shfl_xor((int)sb, d);
      sa %= kAdlerMod;
      sb %= kAdlerMod;
    }
    a = (a + sa) % kAdlerMod;
    b = (b + sb) % kAdlerMod;
    run += (uint32_t)__shfl((int)incl, 63);
  }
  if (l == 0) {
    uint8_t* o = reinterpret_cast<uint8_t*>(bk.dst);
    o[0] = 0x78;
    o[1] = 0x9C;
    uint8_t* t = o + run;
    t[0] = 0x01;  // final empty stored block
    t[1] = 0x00;
    t[2] = 0x00;
    t[3] = 0xFF;
    t[4] = 0xFF;
    t[5] = (uint8_t)(b >> 8);
    t[6] = (uint8_t)b;
    t[7] = (uint8_t)(a >> 8);
    t[8] = (uint8_t)a;
    out_len[c] = run + 9;
  }
}

extern "C" __global__ __launch_bounds__(512) void hbx_k7_deflate_write(uint32_t nseg,
                                                                        const hbxz::SegInfo* __restrict__ info,
                                                                        const uint32_t* __restrict__ scratch,
                                                                        const uint64_t* __restrict__ seg_off) {
  using namespace hbxz;
  __shared__ uint32_t img[kImgWords + 2];
  const uint32_t g = blockIdx.x;
  if (g >= nseg) return;
  const uint32_t t = threadIdx.x;
  const uint32_t nbytes = info[g].bytes;
  const uint32_t* slot = scratch + (uint64_t)g * kImgWords;
  for (uint32_t k = t; k < kImgWords + 2u; k += kThreads) img[k] = k < (nbytes + 3u) / 4u ? slot[k] : 0u;
  __syncthreads();
  // image [0, nbytes) -> the stream at byte address D
  uint8_t* D = reinterpret_cast<uint8_t*>(seg_off[g]);
  const uint32_t lead = (uint32_t)((4u - (reinterpret_cast<uint64_t>(D) & 3u)) & 3u);
  const uint32_t head = min(lead, nbytes);
  const uint8_t* ob = reinterpret_cast<const uint8_t*>(img);
  if (t < head) D[t] = ob[t];
  const uint32_t nw = (nbytes - head) >> 2;
  uint32_t* Dw = reinterpret_cast<uint32_t*>(D + head);
  for (uint32_t k = t; k < nw; k += kThreads) Dw[k] = lds4(img, head + 4u * k);
  const uint32_t done = head + 4u * nw;
  if (t < nbytes - done) D[done + t] = ob[done + t];
}

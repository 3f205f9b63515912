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
// Layout of one block's stream (one workgroup per 32 KiB segment; segments
// are parsed independently, so there is no serial dependence between them):
//
//   78 9C | piece | piece | ... | 01 00 00 FF FF | adler32 (BE)
//
//   piece = one non-final dynamic-Huffman block (BTYPE 10) of the LZ77 tokens
//           of a group of up to four consecutive segments under one code
//           (round 4), or of one segment under its own fixed or dynamic code,
//           closed by an empty stored block (a sync flush: 3 zero bits, pad,
//           00 00 FF FF) so the piece ends on a byte boundary; or, if that is
//           not smaller, one non-final stored block (00 | LEN | ~LEN | data).
//           Matches may reach back into the 32 KiB of the block before the
//           segment (its history; the inflater's window holds it).
//
// K7e hbx_k7_deflate_entropy per segment: incompressible early-out (stored),
//                           Adler partials
// K7a hbx_k7_deflate_size   per parsed segment: LZ77 parse; tokens, ranges
//                           and symbol counts into its scratch slot
// K7h hbx_k7_deflate_code   per parsed segment: the group's (or its own)
//                           code, its image into the slot, its size and mode
// K7s hbx_k7_deflate_plan   per block: piece offsets, header, trailer with
//                           the combined Adler-32, stream length
// K7b hbx_k7_deflate_write  per piece: the image (or the group's members'
//                           images, or the source bytes) to the stream
//
// The LZ77 parse (one 1024-thread workgroup per 32 KiB segment):
//   1. candidates, in position order.  The 32 KiB of the block before the
//      segment (its history) are inserted first, then round r covers
//      segment positions 512r..512r+511, two adjacent threads per position
//      (eight bucket entries each, the better of the two kept).  A 2048-bucket
//      hash table of 4-byte prefixes keeps each bucket's 16 latest positions
//      (a 16-bit counter per bucket picks the slot; one barrier per round,
//      so a slot may already hold a later position of the same round, which
//      is skipped).  Each position keeps the longest verified match among its
//      <= 16 candidates within 32 KiB, nearest first on a tie, and drops a
//      4-byte one farther than kFar4: its distance (u16) and length (u8) go
//      to the segment's scratch slot, because the table and 96 KiB of
//      per-position results do not fit the LDS together; they come back into
//      the table's and the history's LDS once the table is done.
//   2. the parse, greedy with three-step lazy matching (a match at p+k longer
//      than the one at p by k or more, k = 1..3, defers p as a literal; zlib's
//      lazy matching looks one step ahead), from the stored lengths alone (no byte
//      compares).  Thread t < 512 owns the 64-byte range [64t, 64t+64) but a
//      match may run past its end (up to 258 bytes), and the next thread then
//      starts where it ended: every thread first parses from its range start
//      ("dry", no writes), the ends are handed on, and threads whose start
//      moved parse again, until no start moves (greedy parses resynchronise
//      within a few tokens, so this takes one or two rounds; after 8 the
//      starts are made ascending and each thread's final parse is clipped to
//      its successor's start, which keeps the stream exact either way).  The
//      final parse records the tokens, symbol frequencies and fixed-code bits;
//   3. (K7h) after a workgroup prefix sum of the bit counts, the tokens are
//      emitted (ds_or) into the image, if that is smaller than stored; a
//      stored segment is copied by K7b from the source.
// Zipf text of tools/bench_deflate.py: 0.3108 of its size at 16.0 GB/s (zlib
// -6: 0.3114; 0.3115 with a code per segment; round 3: 0.327 at 16.0 GB/s
// with 8 ways of 2,048 buckets, 16 KiB of history and one-step lazy matching;
// 8 ways of 4,096 buckets here: 0.3162 at 23.1 GB/s).  tools/k7model/
// k7model.c models the variants.  LDS: K7a 141, K7h 108 of the CU's 160 KiB.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "hbx_device.h"  // DPP wave scans

namespace hbxz {

constexpr uint32_t kSeg = 32768;  // bytes per segment (one workgroup)
constexpr uint32_t kThreads = 1024;  // K7a
constexpr uint32_t kWaves = kThreads / 64;
constexpr uint32_t kPair = 2;                // threads per position in the candidate rounds
constexpr uint32_t kRound = kThreads / kPair;  // positions per candidate round
constexpr uint32_t kParse = 512;            // parse ranges (threads t >= kParse have empty ones)
constexpr uint32_t kSub = kSeg / kParse;    // 64 bytes per range
constexpr uint32_t kWThreads = 512;         // K7b
constexpr uint32_t kHashBits = 11;
constexpr uint32_t kWays = 16;                // positions kept per bucket (16-bit entries)
constexpr uint32_t kHist = 32768;             // history bytes before a segment (within its block)
constexpr uint32_t kHistWords = kHist / 4;
constexpr uint32_t kWindow = 32768;           // deflate's largest distance
constexpr uint32_t kParseRounds = 8;          // bound on the start hand-off rounds
constexpr uint32_t kRepSet = 2048;            // slots of the early-out's repeat sample set
constexpr uint32_t kDataWords = kSeg / 4 + 8;        // + slack for the 16-byte reads past the end
constexpr uint32_t kDataPhys = (kDataWords + 15u) & ~15u;  // whole swizzle groups
// The candidate array lives in LDS with one pad dword per parse range (kSub/2
// candidate dwords): thread t's range starts kSub bytes after thread t-1's,
// which without padding puts the 64 lanes of a wave on a few banks.  The
// window's words are XOR-swizzled instead (sw below), which keeps 8-byte pairs
// whole for ds_read_b64.
constexpr uint32_t kCdShift = 31 - __builtin_clz(kSub / 2);
constexpr uint32_t kCdPhys = (kSeg / 2 + (kSeg / 2 >> kCdShift)) * 2;  // u16 slots
constexpr uint32_t kImgWords = (kSeg + 16) / 4 + 4;  // stored image (5 + kSeg) or a smaller fixed one
// hash table: 2048 x 16 u16 entries (window position + 1), then 2048 u16
// counters, in the region that holds the candidate distances after step 1
constexpr uint32_t kTabWords = (1u << kHashBits) * kWays / 2 + (1u << kHashBits) / 2;
// scratch bytes per segment: the candidate distances (u16 per position) and
// their match lengths (u8 per position, length - 3, 0 = none) between steps 1
// and 2, then the coded image
constexpr uint32_t kSlot = 3u * kSeg;
constexpr uint32_t kSlotLens = 2u * kSeg;  // byte offset of the lengths
static_assert(kSlot >= kImgWords * 4u, "the image fits its slot");
// after the parse (K7a -> K7h), in words: the tokens at 0 (later the image),
// each thread's token range start, end and fixed-code bits, the symbol
// counts (litlen 0..285 and distances at 288..317, as the code lengths are
// indexed; then the fixed-code and extra bit totals), and K7h's placement of
// the image in its group's piece (byte offset, bytes, members)
constexpr uint32_t kSlotThr = (kCdPhys / 2u + 15u) & ~15u;
constexpr uint32_t kSlotRec = kSlotThr + 3u * 1024u;
constexpr uint32_t kRecWords = 322;
constexpr uint32_t kSlotMeta = kSlotRec + kRecWords + 2u;
static_assert((kSlotMeta + 4u) * 4u <= kSlot, "the hand-off fits the slot");
// kGroup consecutive segments of a block share one dynamic code (one header,
// one end of block and sync flush) when that is smaller; K7b assembles the
// group's piece from the members' images
constexpr uint32_t kGroup = 4;
constexpr uint32_t kTabLds = kTabWords > kCdPhys / 2u ? kTabWords : kCdPhys / 2u;  // table, then distances
// window positions + 1 are u16 entries, and a bucket's u16 insert counter
// never carries into its neighbour's
static_assert(kHist + kSeg <= 65536u, "window positions fit 16 bits");
constexpr uint32_t kAdlerMod = 65521;
constexpr uint32_t kLazy = 32;  // no look-ahead past a match this long
constexpr uint32_t kFar4 = 1024;  // farthest 4-byte match kept

struct SegInfo {
  uint32_t bytes;  // coded bytes of the segment (stored or fixed image)
  uint32_t mode;   // 1 fixed, 2 dynamic Huffman; 3/6 stored (from the source; K7e/K7h); 4/5 group head/member; 0xFF parse
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
// Window words in LDS: word k at k ^ 2 * ((k / 16) % 8), a permutation inside
// each 16-word group that keeps every even/odd pair together (ds_read_b64)
// and puts words 16 apart (the starts of neighbouring parse ranges, the
// literal reads of the recording pass) on different banks.  History and
// segment share it (the segment starts at word kHistWords, a multiple of 128).
__device__ __forceinline__ uint32_t sw(uint32_t k) { return k ^ (((k >> 4) & 7u) << 1); }
// 4 bytes at byte p of the padded segment
__device__ __forceinline__ uint32_t seg4(const uint32_t* w, uint32_t p) {
  const uint32_t i = p >> 2;
  return __builtin_amdgcn_alignbyte(w[sw(i + 1u)], w[sw(i)], p & 3u);
}
__device__ __forceinline__ uint32_t cphys(uint32_t p) {
  const uint32_t wd = p >> 1;
  return 2u * (wd + (wd >> kCdShift)) + (p & 1u);
}

// The match lengths in LDS (over the history's words once step 1 is done):
// byte p of word (p / 4) XOR-swizzled within each 16-word group, so the 64
// lanes of a wave, whose ranges start 64 bytes apart, hit different banks.
__device__ __forceinline__ uint32_t lphys(uint32_t p) {
  const uint32_t w = p >> 2;
  return ((w ^ ((w >> 4) & 15u)) << 2) | (p & 3u);
}

__device__ __forceinline__ uint32_t zhash(uint32_t x) { return (x * 0x9E3779B1u) >> (32 - kHashBits); }
// K7e's content-defined sample (1 in 64 four-byte values)
__device__ __forceinline__ bool sampled(uint32_t x) { return ((x * 0x9E3779B1u) >> 21 & 63u) == 0u; }

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
  for (uint32_t k = threadIdx.x; k < kDataWords; k += kThreads) data[sw(k)] = k < nw ? base[k] : 0u;
}

// Window word i: the history's words first, then the segment's, one LDS
// array (data == hist + kHistWords); hw = history words present (0 or
// kHistWords), so window word i is array word kHistWords - hw + i.
__device__ __forceinline__ uint32_t wword(const uint32_t* hist, const uint32_t* data, uint32_t hw, uint32_t i) {
  (void)data;
  return hist[sw(kHistWords - hw + i)];
}
// 4 bytes at window byte b (window position + sh)
__device__ __forceinline__ uint32_t win4(const uint32_t* hist, const uint32_t* data, uint32_t hw, uint32_t b) {
  const uint32_t i = b >> 2;
  return __builtin_amdgcn_alignbyte(wword(hist, data, hw, i + 1u), wword(hist, data, hw, i), b & 3u);
}

// 16 bytes from byte r of array word i (base 8-byte aligned), as 4 dwords:
// three ds_read_b64 of the aligned pairs around them (a random b64 costs the
// LDS about what a random b32 does, so 3 loads instead of 5)
__device__ __forceinline__ void load16(const uint32_t* base, uint32_t i, uint32_t r, uint32_t (&c)[4]) {
  const uint32_t i0 = i & ~1u;
  uint32_t v[6];
#pragma unroll
  for (uint32_t j = 0; j < 3u; j++) {
    const uint2 x = *reinterpret_cast<const uint2*>(base + sw(i0 + 2u * j));
    v[2 * j] = x.x;
    v[2 * j + 1] = x.y;
  }
  // (a mask select: written as v[j + odd] the compiler indexes the array in scratch)
  const uint32_t m = 0u - (i & 1u);
  uint32_t w[5];
#pragma unroll
  for (int j = 0; j < 5; j++) w[j] = (v[j] & ~m) | (v[j + 1] & m);
#pragma unroll
  for (int j = 0; j < 4; j++) c[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], r);
}
// 16 bytes at segment byte b (position + sh) / window byte b
__device__ __forceinline__ void seg16(const uint32_t* data, uint32_t b, uint32_t (&c)[4]) {
  load16(data, b >> 2, b & 3u, c);
}
__device__ __forceinline__ void win16(const uint32_t* hist, const uint32_t* data, uint32_t hw, uint32_t b,
                                      uint32_t (&c)[4]) {
  (void)data;
  load16(hist, kHistWords - hw + (b >> 2), b & 3u, c);
}
// leading equal bytes of two 16-byte strings (0..16)
__device__ __forceinline__ uint32_t eq16(const uint32_t (&a)[4], const uint32_t (&b)[4]) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t d = a[j] ^ b[j];
    if (d) return 4u * (uint32_t)j + ((uint32_t)__builtin_ctz(d) >> 3);
  }
  return 16u;
}

// Common prefix length of the segment string at p and the window string at
// window position q (q < p + hl), at most limit: the first 16 bytes with
// independent loads, then 4 bytes per compare (matches past 16 are rare).
__device__ __forceinline__ uint32_t match_len(const uint32_t* hist, const uint32_t* data, uint32_t hw,
                                              uint32_t sh, uint32_t p, uint32_t q, uint32_t limit) {
  uint32_t a[4], b[4];
  seg16(data, p + sh, a);
  win16(hist, data, hw, q + sh, b);
  uint32_t len = eq16(a, b);
  if (len < 16u) return min(len, limit);
  while (len < limit) {
    const uint32_t dlt = seg4(data, p + len + sh) ^ win4(hist, data, hw, q + len + sh);
    if (dlt) {
      len += (uint32_t)__builtin_ctz(dlt) >> 3;
      break;
    }
    len += 4u;
  }
  return min(len, limit);
}

// Length and distance symbols (RFC 1951 §3.2.5): symbol, extra-bit count,
// extra-bit value.
__device__ __forceinline__ void len_sym(uint32_t len, uint32_t& sym, uint32_t& ne, uint32_t& ex) {
  ne = 0u;
  ex = 0u;
  if (len <= 10u) {
    sym = 254u + len;
  } else if (len == 258u) {
    sym = 285u;
  } else {
    const uint32_t l = len - 3u;
    ne = 31u - __builtin_clz(l) - 2u;
    sym = 257u + 4u * (ne + 1u) + ((l >> ne) & 3u);
    ex = l & ((1u << ne) - 1u);
  }
}
__device__ __forceinline__ void dist_sym(uint32_t dist, uint32_t& sym, uint32_t& ne, uint32_t& ex) {
  const uint32_t d = dist - 1u;
  ne = 0u;
  ex = 0u;
  if (d < 4u) {
    sym = d;
  } else {
    ne = 31u - __builtin_clz(d) - 1u;
    sym = 2u * (ne + 1u) + ((d >> ne) & 1u);
    ex = d & ((1u << ne) - 1u);
  }
}

// Step 2: the greedy parse of one thread, three-step lazy, with the candidate
// distances in `cd` (d = 0: none).  Dry (REC = false): from s while p < rend
// (the thread's range end), matches up to min(258, n - p); returns where the
// last token ends, which may be past rend.  Final (REC = true): from s while
// p < send (the next thread's start), matches clipped to send; the tokens
// overwrite the candidate slots they cover (already consumed): a literal at p
// is 0x8000 | byte in slot p; a match is len in slot p and dist in slot p+1.
// Symbol frequencies go to hll/hd; `bits` = fixed-code bits, `extra` = extra
// bits (the same under any code).  Lookahead to p + 1 .. p + 3 only while
// that is < rend, in both passes, so a converged final parse repeats the dry
// one token for token (and never reads a slot past the thread's own range,
// since its tokens end at or past rend).
// The dry pass also returns its token starts as a mask over the thread's
// 64-byte range (bit i = a token starts at range start + i): a token of one
// byte is a literal, a longer one the match of that length at distance cd[p].
template <bool REC>
__device__ __forceinline__ uint32_t parse(const uint32_t* data, const uint8_t* l8, uint16_t* cd, uint32_t* hll,
                                          uint32_t* hd, uint32_t sh, uint32_t n, uint32_t s, uint32_t rend,
                                          uint32_t send, uint32_t& bits, uint32_t& extra,
                                          uint64_t* starts_mask = nullptr, uint32_t r0 = 0u) {
  const uint32_t stop = REC ? send : rend;
  const uint32_t cap = REC ? send : n;
  // the match at q, at most cap - q long (step 1 measured it up to
  // min(258, n - q); cap <= n, so the clip equals a compare up to the clip)
  auto len_at = [&](uint32_t q) -> uint32_t {
    const uint32_t v = l8[lphys(q)];
    return v ? min(v + 3u, cap - q) : 0u;
  };
  uint32_t p = s, len = 0u, d = 0u;
  bits = 0u;
  extra = 0u;
  bool have = false;  // (len, d) already hold the match at p
  uint64_t mask = 0ull;
  while (p < stop) {
    if (!REC) mask |= 1ull << (p - r0);
    if (!have) {
      d = cd[cphys(p)];
      len = d ? len_at(p) : 0u;
    }
    have = false;
    bool defer = false;
    uint32_t len1 = 0u, d1 = 0u;
    if (len >= 4u && len < kLazy && p + 1u < rend) {
      d1 = cd[cphys(p + 1u)];
      len1 = d1 ? len_at(p + 1u) : 0u;
      defer = len1 > len;  // lazy: p becomes a literal, the longer match starts at p + 1
      // further steps: a match at p + k longer than len + k - 1 also defers
      // p (p + 1 .. p + k - 1 then defer to it in turn)
      if (!defer && p + 2u < rend) defer = len_at(p + 2u) > len + 1u;
      if (!defer && p + 3u < rend) defer = len_at(p + 3u) > len + 2u;
    }
    if (len >= 4u && !defer) {
      if (REC) {
        uint32_t v, nb, sym, ne, ex, ds, dne, dex;
        match_code(len, d, v, nb);
        len_sym(len, sym, ne, ex);
        dist_sym(d, ds, dne, dex);
        atomicAdd(&hll[sym], 1u);
        atomicAdd(&hd[ds], 1u);
        extra += ne + dne;
        bits += nb;
        cd[cphys(p)] = (uint16_t)len;
        cd[cphys(p + 1u)] = (uint16_t)d;
      }
      p += len;
    } else {
      if (REC) {
        const uint32_t b = seg4(data, p + sh) & 0xFFu;
        atomicAdd(&hll[b], 1u);
        bits += b < 144u ? 8u : 9u;
        cd[cphys(p)] = (uint16_t)(0x8000u | b);
      }
      p += 1u;
      if (defer) {
        len = len1;
        d = d1;
        have = true;
      }
    }
  }
  if (!REC && starts_mask) *starts_mask = mask;
  return p;
}

// The recording pass from a dry pass's token starts (the converged case: the
// tokens are the dry pass's, ending at `e`), without recomputing any match.
__device__ __forceinline__ void record_tokens(const uint32_t* data, uint16_t* cd, uint32_t* hll, uint32_t* hd,
                                              uint32_t sh, uint32_t r0, uint64_t mask, uint32_t e,
                                              uint32_t& bits, uint32_t& extra) {
  bits = 0u;
  extra = 0u;
  while (mask) {
    const uint32_t i = (uint32_t)__builtin_ctzll(mask);
    mask &= mask - 1ull;
    const uint32_t p = r0 + i;
    const uint32_t nx = mask ? r0 + (uint32_t)__builtin_ctzll(mask) : e;
    const uint32_t len = nx - p;
    if (len == 1u) {
      const uint32_t b = seg4(data, p + sh) & 0xFFu;
      atomicAdd(&hll[b], 1u);
      bits += b < 144u ? 8u : 9u;
      cd[cphys(p)] = (uint16_t)(0x8000u | b);
    } else {
      const uint32_t d = cd[cphys(p)];
      uint32_t v, nb, sym, ne, ex, ds, dne, dex;
      match_code(len, d, v, nb);
      len_sym(len, sym, ne, ex);
      dist_sym(d, ds, dne, dex);
      atomicAdd(&hll[sym], 1u);
      atomicAdd(&hd[ds], 1u);
      extra += ne + dne;
      bits += nb;
      cd[cphys(p)] = (uint16_t)len;
      cd[cphys(p + 1u)] = (uint16_t)d;
    }
  }
}

__device__ __forceinline__ void emit_bits(uint32_t* img, uint32_t& o, uint32_t v, uint32_t nb) {
  const uint32_t w = o >> 5, s = o & 31u;
  atomicOr(&img[w], v << s);
  if (s + nb > 32u) atomicOr(&img[w + 1u], v >> (32u - s));
  o += nb;
}

// Step 3: walk thread t's tokens with the code tables (entry = reversed code
// | length << 16); EMIT = false returns their bits, EMIT = true writes them.
template <bool EMIT>
__device__ __forceinline__ uint32_t walk_tokens(const uint16_t* cd, const uint32_t* llc, const uint32_t* dcc,
                                                uint32_t* img, uint32_t s, uint32_t send, uint32_t o) {
  uint32_t bits = 0u;
  for (uint32_t p = s; p < send;) {
    const uint32_t v = cd[cphys(p)];
    if (v & 0x8000u) {
      const uint32_t e = llc[v & 0xFFu];
      if (EMIT) emit_bits(img, o, e & 0xFFFFu, e >> 16);
      bits += e >> 16;
      p += 1u;
    } else {
      const uint32_t dist = cd[cphys(p + 1u)];
      uint32_t sym, ne, ex, ds, dne, dex;
      len_sym(v, sym, ne, ex);
      dist_sym(dist, ds, dne, dex);
      const uint32_t e = llc[sym], f = dcc[ds];
      const uint32_t nl = (e >> 16) + ne, nd = (f >> 16) + dne;
      if (EMIT) {
        emit_bits(img, o, (e & 0xFFFFu) | (ex << (e >> 16)), nl);
        emit_bits(img, o, (f & 0xFFFFu) | (dex << (f >> 16)), nd);
      }
      bits += nl + nd;
      p += v;
    }
  }
  return bits;
}

// ---- dynamic Huffman codes (RFC 1951 §3.2.7) -------------------------------
// The two-queue merge of a Huffman tree, for the parallel depth pass: keys
// (freq << 9 | symbol) ascending, leaves 0..m) in key order, internal nodes
// m..2m-1); par[node] = pbase + its parent; leaf first on equal weights.
__device__ void huff_merge(const uint32_t* keys, uint32_t m, uint32_t shift, uint32_t* w, uint32_t* par,
                           uint32_t pbase) {
  constexpr uint32_t kInf = 0xFFFFFFFFu;
  auto leaf = [&](uint32_t i) { return i < m ? ((keys[i] >> 9) >> shift) | 1u : kInf; };
  uint32_t i = 0u, j = m, wi = leaf(0u), wj = kInf;
  for (uint32_t k = m; k < 2u * m - 1u; k++) {
    uint32_t a, b, wa, wb;
    if (wi <= wj) { a = i++; wa = wi; wi = leaf(i); } else { a = j++; wa = wj; wj = j < k ? w[j] : kInf; }
    if (wi <= wj) { b = i++; wb = wi; wi = leaf(i); } else { b = j++; wb = wj; wj = j < k ? w[j] : kInf; }
    const uint32_t s = wa + wb;
    w[k] = s;
    if (j == k) wj = s;  // the internal queue was empty: the new node heads it
    par[a] = pbase + k;
    par[b] = pbase + k;
  }
}

// The run-length code of one run of `run` equal code lengths `cur`, as
// huff header symbols (16 repeat 3-6, 17 zeros 3-10, 18 zeros 11-138), in
// zlib's order.  With EMIT they go to out[] and their counts into f[].
template <bool EMIT>
__device__ __forceinline__ uint32_t rle_runs(uint32_t cur, uint32_t r, uint32_t* out, uint32_t* f) {
  uint32_t nr = 0u;
  auto put = [&](uint32_t sym) {
    if (EMIT) {
      out[nr] = sym;
      atomicAdd(&f[sym & 31u], 1u);
    }
    nr++;
  };
  if (cur == 0u) {
    while (r >= 11u) {
      const uint32_t q = min(r, 138u);
      put(18u | ((q - 11u) << 8));
      r -= q;
    }
    if (r >= 3u) {
      put(17u | ((r - 3u) << 8));
      r = 0u;
    }
  } else {
    put(cur);
    r--;
    while (r >= 3u) {
      const uint32_t q = min(r, 6u);
      put(16u | ((q - 3u) << 8));
      r -= q;
    }
  }
  while (r > 0u) {
    put(cur);
    r--;
  }
  return nr;
}

// Order of the code-length code lengths in the header (RFC 1951 §3.2.7).
__device__ const uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// position of each code-length symbol in kClOrder
__device__ const uint8_t kClPos[19] = {3, 17, 15, 13, 11, 9, 7, 5, 4, 6, 8, 10, 12, 14, 16, 18, 0, 1, 2};

__device__ __forceinline__ uint64_t wave_min64(uint64_t v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t o = ((uint64_t)(uint32_t)__shfl_xor((int)(v >> 32), d) << 32) | (uint32_t)__shfl_xor((int)(uint32_t)v, d);
    v = o < v ? o : v;
  }
  return v;
}
__device__ __forceinline__ uint32_t wave_max32(uint32_t v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, d));
  return v;
}

// The code-length code (<= 19 symbols, lengths <= 7) built by one wave, lane
// l = symbol l, the tree's internal nodes on lanes 19.. as they are made:
// each merge takes the two smallest available nodes by (weight, leaf before
// internal, key) with two wave minimum reductions, depths by pointer jumping
// over the parent lanes; a tree deeper than 7 is rebuilt from halved
// frequencies (always a complete code).  Then the canonical codes (RFC 1951
// §3.2.2) and HCLEN.  All 64 lanes call it; f = the lane's frequency (0 past
// 18).  Writes cll[0..19), clc[0..19) and returns HCLEN.
__device__ uint32_t cl_code(uint32_t f, uint8_t* cll, uint32_t* clc) {
  constexpr uint64_t kNone = ~0ull;
  const uint32_t l = threadIdx.x & 63u;
  const bool leaf = l < 19u && f != 0u;
  const uint64_t nz = __builtin_amdgcn_ballot_w64(leaf);
  const uint32_t mc = (uint32_t)__builtin_popcountll(nz);
  uint32_t len = 0u;
  if (mc == 1u) {  // one used symbol: two codes of one bit (RFC 1951 §3.2.7)
    const uint32_t x = (uint32_t)__builtin_ctzll(nz);
    len = l == x || l == (x ? 0u : 1u) ? 1u : 0u;
  } else {
    for (uint32_t shift = 0;; shift++) {
      uint32_t wgt = leaf ? (f >> shift) | 1u : 0u, par = l;
      bool avail = leaf;
      for (uint32_t k = 0; k + 1u < mc; k++) {
        // sortable: weight | internal | key (leaves: freq << 9 | symbol; internal: creation index) | lane
        const uint64_t key = ((uint64_t)wgt << 32) | ((uint64_t)(l >= 19u) << 31) |
                             ((uint64_t)(l < 19u ? (f << 9) | l : l - 19u) << 6) | l;
        const uint64_t m1 = wave_min64(avail ? key : kNone);
        const uint32_t a = (uint32_t)(m1 & 63u);
        const uint64_t m2 = wave_min64(avail && l != a ? key : kNone);
        const uint32_t b = (uint32_t)(m2 & 63u);
        const uint32_t nn = 19u + k;
        if (l == a || l == b) {
          par = nn;
          avail = false;
        }
        if (l == nn) {
          wgt = (uint32_t)(m1 >> 32) + (uint32_t)(m2 >> 32);
          avail = true;
        }
      }
      // depth = steps to the root (the last node made, its own parent)
      uint32_t d = par != l ? 1u : 0u, p = par;
#pragma unroll
      for (int r = 0; r < 6; r++) {  // depth <= 18 < 2^6
        const uint32_t dp = (uint32_t)__shfl((int)d, (int)p), pp = (uint32_t)__shfl((int)p, (int)p);
        d += dp;
        p = pp;
      }
      len = leaf ? d : 0u;
      if (wave_max32(len) <= 7u) break;
    }
  }
  // canonical codes: the first code of each length, then the rank among the
  // same length's smaller symbols
  uint32_t code = 0u, first = 0u, prev = 0u;
  for (uint32_t bl = 1; bl <= 7u; bl++) {
    code = (code + prev) << 1;
    if (len == bl) first = code;
    prev = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(l < 19u && len == bl));
  }
  uint32_t rank = 0u;
  for (uint32_t bl = 1; bl <= 7u; bl++) {
    const uint64_t mb = __builtin_amdgcn_ballot_w64(l < 19u && len == bl);
    if (len == bl) rank = (uint32_t)__builtin_popcountll(mb & ((1ull << l) - 1ull));
  }
  if (l < 19u) {
    cll[l] = (uint8_t)len;
    clc[l] = len ? rev(first + rank, len) | (len << 16) : 0u;
  }
  return max(4u, wave_max32(l < 19u && len ? (uint32_t)kClPos[l] + 1u : 0u));
}

__device__ __forceinline__ uint32_t wg_incl_sum(uint32_t x, uint32_t* wsum, uint32_t& tot) {
  const uint32_t l = threadIdx.x & 63u, w = threadIdx.x >> 6;
  x = hbx::wave_incl_sum(x);  // DPP
  if (l == 63u) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0u;
  for (uint32_t k = 0; k < w; k++) before += wsum[k];
  tot = 0u;
  for (uint32_t k = 0; k < kWaves; k++) tot += wsum[k];
  __syncthreads();
  return before + x;
}

// Workgroup inclusive prefix sum of x[0] and totals of x[0..N) in one pair
// of barriers (wsum: N * kWaves words).
template <int N>
__device__ __forceinline__ uint32_t wg_sums(const uint32_t (&x)[N], uint32_t* wsum, uint32_t (&tot)[N]) {
  const uint32_t l = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t v = hbx::wave_incl_sum(x[0]);  // DPP; lane 63 holds each wave total
  uint32_t r[N];
  r[0] = v;
#pragma unroll
  for (int i = 1; i < N; i++) r[i] = hbx::wave_incl_sum(x[i]);
  if (l == 63u) {
#pragma unroll
    for (int i = 0; i < N; i++) wsum[i * kWaves + w] = r[i];
  }
  __syncthreads();
  uint32_t before = 0u;
  for (uint32_t k = 0; k < w; k++) before += wsum[k];
#pragma unroll
  for (int i = 0; i < N; i++) {
    uint32_t t = 0u;
    for (uint32_t k = 0; k < kWaves; k++) t += wsum[i * kWaves + k];
    tot[i] = t;
  }
  __syncthreads();
  return before + v;
}

}  // namespace hbxz

// Diagnostics (tools/ubench/k7_phases.hip builds with HBX_K7_PROBE=1): thread
// 0 of each workgroup stamps s_memtime at the phase boundaries.
#ifndef HBX_K7_PROBE
#define HBX_K7_PROBE 0
#endif
#if HBX_K7_PROBE
__device__ unsigned long long hbx_k7_probe[1 << 20];
#define K7P(i) \
  if (threadIdx.x == 0 && blockIdx.x < (1u << 16)) hbx_k7_probe[16u * blockIdx.x + (i)] = __builtin_amdgcn_s_memtime()
#else
#define K7P(i)
#endif

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

namespace hbxz {
constexpr uint32_t kModeSrcStored = 3u;    // SegInfo.mode: stored, K7b copies the bytes from the source
constexpr uint32_t kModeParse = 0xFFu;     // SegInfo.mode set by K7e: K7a decides
constexpr uint32_t kModeGroupHead = 4u;    // first segment of a shared-code group: bytes = the group's piece
constexpr uint32_t kModeGroupMember = 5u;  // a later member: its bits are in the head's piece (bytes = 0)
// K7h's own "stored" decision.  K7b treats it as kModeSrcStored, but it is a
// value of its own: K7h reads its group siblings' info[].mode (was the member
// stored by K7e?) while those siblings' K7h may already be overwriting it, so
// K7h never writes kModeSrcStored and "!= kModeSrcStored" keeps meaning "not
// stored by K7e" whatever a sibling has written by then (advisor r04).
constexpr uint32_t kModeOwnStored = 6u;
constexpr uint32_t kEThreads = 256;
}  // namespace hbxz

// K7e, the incompressible early-out on its own (round 4): one 256-thread
// workgroup per segment and 9 KiB of LDS (six per CU instead of K7a's one),
// reading the segment straight from global memory.  The same rule as K7a's
// step 0: a segment of >= 4096 bytes whose order-0 entropy is >= 7.97 bits
// per byte and whose content-sampled 4-byte values never repeat is stored:
// info[g] = {5 + n, kModeSrcStored, Adler partials}, and K7b copies its bytes
// from the source (no image in the scratch).  Every other segment gets
// kModeParse and goes through K7a.  (Random data: K7a's one 162 KB workgroup
// per CU ran the early-out phases back to back, 241 GB/s.)
extern "C" __global__ __launch_bounds__(256) void hbx_k7_deflate_entropy(const hbxz::ZBlock* __restrict__ blocks,
                                                                         uint32_t nb, uint32_t nseg,
                                                                         hbxz::SegInfo* __restrict__ info) {
  using namespace hbxz;
  __shared__ uint32_t cnt[256];
  __shared__ uint32_t set[kRepSet];
  __shared__ uint32_t wred[kEThreads / 64][3];
  __shared__ uint32_t rep_any;
  const uint32_t g = blockIdx.x;
  if (g >= nseg) return;
  const ZBlock bk = blocks[zblock_of(blocks, nb, g)];
  const uint32_t s = g - bk.seg0;
  const uint64_t off = (uint64_t)s * kSeg;
  const uint32_t n = (uint32_t)min((uint64_t)kSeg, bk.len - off);
  const uint32_t t = threadIdx.x;
  const uint64_t a = bk.src + off;
  const uint32_t sh = (uint32_t)(a & 3u);
  const uint32_t* base = reinterpret_cast<const uint32_t*>(a - sh);
  const uint32_t nw = (n + sh + 3u) >> 2;  // words holding a byte of the segment
  for (uint32_t k = t; k < 256u; k += kEThreads) cnt[k] = 0u;
  for (uint32_t k = t; k < kRepSet; k += kEThreads) set[k] = 0u;
  if (t == 0) rep_any = 0u;
  __syncthreads();
  auto sample = [&](uint32_t x) -> bool {  // (K7a's step 0)
    if (!sampled(x)) return false;
    const uint32_t key = x + 1u ? x + 1u : 1u;
    const uint32_t i0 = (x * 0x85EBCA6Bu) >> (32 - 11);
    for (uint32_t r = 0; r < 8u; r++) {
      const uint32_t old = atomicCAS(&set[(i0 + r) & (kRepSet - 1u)], 0u, key);
      if (old == 0u) return false;
      if (old == key) return true;
    }
    return false;
  };
  // thread t: aligned words k = t, t + 256, ...; positions p = 4k + j - sh
  uint64_t A = 0ull, J = 0ull;
  bool rep = false;
  for (uint32_t k = t; k < nw; k += kEThreads) {
    const uint32_t w0 = base[k], w1 = k + 1u < nw ? base[k + 1u] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < 4u; j++) {
      const int64_t p = 4ll * k + j - sh;
      if (p < 0 || p >= (int64_t)n) continue;
      const uint32_t x = __builtin_amdgcn_alignbyte(w1, w0, j);
      const uint32_t b = x & 0xFFu;
      atomicAdd(&cnt[b], 1u);
      A += b;
      J += (uint64_t)p * b;
      if ((uint32_t)p + 4u <= n) rep |= sample(x);
    }
  }
  // the history's samples too (round 4): a segment whose repeats lie only in
  // the 32 KiB before it (in its block) is parsed, not stored, since K7a's
  // matches reach there.  Only the history's word-aligned positions: a
  // repeated stretch of a few hundred bytes still holds several sampled
  // positions at each of the four alignments, and the pass costs a quarter
  // (random data 690 -> 440 GB/s sampling every position); a repeat inside
  // the history alone only costs a parse
  if (s) {
    const uint32_t* hb = base - kHist / 4u;  // the aligned base was the segment's start rounded down
    for (uint32_t k = t; k < kHist / 4u; k += kEThreads) rep |= sample(hb[k]);
  }
  if (rep) rep_any = 1u;
  __syncthreads();
  // per-symbol bits rounded, summed over the workgroup (K7a's formula)
  const uint32_t c = cnt[t];
  uint32_t bits = c ? (uint32_t)((float)c * (__log2f((float)n) - __log2f((float)c)) + 0.5f) : 0u;
  uint64_t A64 = A, J64 = J;
  for (int d = 32; d >= 1; d >>= 1) {
    bits += (uint32_t)__shfl_xor((int)bits, d);
    A64 += (unsigned long long)__shfl_xor((long long)A64, d);
    J64 += (unsigned long long)__shfl_xor((long long)J64, d);
  }
  __shared__ unsigned long long wad[kEThreads / 64][2];
  if ((t & 63u) == 0u) {
    wred[t >> 6][0] = bits;
    wad[t >> 6][0] = A64;
    wad[t >> 6][1] = J64;
  }
  __syncthreads();
  if (t == 0) {
    uint32_t hsum = 0u;
    unsigned long long As = 0, Js = 0;
    for (uint32_t w = 0; w < kEThreads / 64; w++) {
      hsum += wred[w][0];
      As += wad[w][0];
      Js += wad[w][1];
    }
    // (every segment's Adler partials come from here; K7a no longer sums them)
    const bool incompressible = n >= 4096u && (float)hsum >= 7.97f * (float)n && rep_any == 0u;
    SegInfo si;
    si.mode = incompressible ? kModeSrcStored : kModeParse;
    si.bytes = 5u + n;
    si.a = (uint32_t)(As % kAdlerMod);
    si.b = (uint32_t)(((unsigned long long)n * As - Js) % kAdlerMod);
    info[g] = si;
  }
}

extern "C" __global__ __launch_bounds__(hbxz::kThreads) void hbx_k7_deflate_size(const hbxz::ZBlock* __restrict__ blocks,
                                                                       uint32_t nb, uint32_t nseg,
                                                                       hbxz::SegInfo* __restrict__ info,
                                                                       uint32_t* __restrict__ scratch) {
  using namespace hbxz;
  // history words, then the segment's; after the parse, the Huffman scratch
  // and then the coded image
  __shared__ __attribute__((aligned(16))) uint32_t win[kHistWords + kDataPhys];
  uint32_t* const hist = win;
  uint32_t* const data = win + kHistWords;
  // the hash table (step 1), then the candidate distances (steps 2-3)
  __shared__ uint32_t tab[kTabLds];
  uint16_t* const cd = reinterpret_cast<uint16_t*>(tab);
  __shared__ uint32_t starts[kThreads + 1];  // each thread's parse start (step 2)
  __shared__ uint32_t wsum4[4 * kWaves];
  __shared__ uint32_t hll[288], hd[32];
  const uint32_t g = blockIdx.x;
  // K7e ran first: its stored segments are done (the early-out of step 0 in
  // rounds 1-3 lives there now), every other segment is parsed
  if (g >= nseg || info[g].mode == kModeSrcStored) return;
  K7P(0);
  const ZBlock bk = blocks[zblock_of(blocks, nb, g)];
  const uint32_t s = g - bk.seg0;
  const uint64_t off = (uint64_t)s * kSeg;
  const uint32_t n = (uint32_t)min((uint64_t)kSeg, bk.len - off);
  const uint32_t t = threadIdx.x;
  uint32_t sh;
  const uint8_t* seg_src = reinterpret_cast<const uint8_t*>(bk.src) + off;
  load_segment(data, seg_src, n, sh);
  // history: the kHist bytes of the block before this segment (word j holds
  // window bytes [4j - sh, 4j - sh + 4), like the segment's words); segment
  // s >= 1 starts kSeg = kHist bytes into its block
  static_assert(kHist <= kSeg, "a segment's history lies in its block");
  const uint32_t hl = s ? kHist : 0u, hw = hl / 4u;
  if (hl) {
    const uint32_t* hb = reinterpret_cast<const uint32_t*>(seg_src - sh - hl);
    for (uint32_t k = t; k < hw; k += kThreads) hist[sw(k)] = hb[k];
  }
  for (uint32_t k = t; k < kTabWords; k += kThreads) tab[k] = 0u;
  for (uint32_t k = t; k < 288u; k += kThreads) hll[k] = k == 256u ? 1u : 0u;  // EOB once
  for (uint32_t k = t; k < 32u; k += kThreads) hd[k] = 0u;
  __syncthreads();

  K7P(1);
  uint32_t fbits = 0u;
  uint32_t p_s = 0u, p_e = 0u;  // this thread's tokens: positions [p_s, p_e)
  // this segment's scratch slot: the candidate distances, later the image
  uint32_t* const slot = scratch + (uint64_t)g * (kSlot / 4u);
  uint16_t* const cdg = reinterpret_cast<uint16_t*>(slot);
  uint8_t* const lg = reinterpret_cast<uint8_t*>(slot) + kSlotLens;
  uint8_t* const l8 = reinterpret_cast<uint8_t*>(hist);  // the lengths, after step 1
  {
    // 1. candidates in position order + Adler partials.  tab16[h*kWays + k]:
    //    window position + 1 of bucket h's k-th entry; cnt16[h]: inserts
    //    so far (the slot of the next one, mod kWays).  Each position's candidate
    //    distance goes to the slot in global memory (the table and the 64 KiB
    //    of distances do not fit the LDS together) and comes back into the
    //    table's LDS once the table is done.
    uint16_t* tab16 = reinterpret_cast<uint16_t*>(tab);
    uint32_t* cnt = tab + (1u << kHashBits) * kWays / 2u;
    auto insert = [&](uint32_t w, uint32_t h) {
      const uint32_t sft = 16u * (h & 1u);
      const uint32_t k = (atomicAdd(&cnt[h >> 1], 1u << sft) >> sft) & (kWays - 1u);
      tab16[h * kWays + k] = (uint16_t)(w + 1u);
    };
    for (uint32_t r = 0; r < hl / kThreads; r++) {  // the history: inserts only, kThreads per round
      const uint32_t w = kThreads * r + t;
      if (w + 4u <= hl + n) insert(w, zhash(win4(hist, data, hw, w + sh)));
      __syncthreads();
    }
    K7P(2);
    // kPair threads per position (adjacent lanes), each over kWays / kPair
    // of the bucket's entries; the best (longest, then nearest) is combined
    // across the pair, the same choice as one thread over all of them
    constexpr uint32_t kMine = kWays / kPair;
    static_assert(kMine == 4u || kMine == 8u, "one 8- or 16-byte load of a thread's entries");
    const uint32_t part = t % kPair;
    // a position's first 16 bytes are loaded one round ahead (the segment's
    // words do not change in step 1), so a round's critical path starts at
    // the bucket read
    uint32_t curn[4];
    seg16(data, t / kPair + sh, curn);
    for (uint32_t r = 0; r < kSeg / kRound; r++) {
      const uint32_t p = kRound * r + t / kPair;
      const uint32_t w = p + hl;
      const uint32_t cur[4] = {curn[0], curn[1], curn[2], curn[3]};
      const uint32_t x = cur[0];
      const bool live = p + 4u <= n;
      const uint32_t h = zhash(x);
      uint32_t best = 0u, bl = 0u;
      if (live) {
        uint32_t cs[kMine / 2];
        if constexpr (kMine == 8u) {
          const uint4 c = *reinterpret_cast<const uint4*>(&tab16[h * kWays + kMine * part]);
          cs[0] = c.x;
          cs[1] = c.y;
          cs[2] = c.z;
          cs[3] = c.w;
        } else {
          const uint2 c = *reinterpret_cast<const uint2*>(&tab16[h * kWays + kMine * part]);
          cs[0] = c.x;
          cs[1] = c.y;
        }
        // this position goes into the table now (the pair's bucket reads came
        // first in the wave's LDS order): its latency overlaps the compares;
        // later positions of the round may see it, earlier ones skip it
        if (part == 0u) insert(w, h);
        const uint32_t lim = min(258u, n - p);
        // the candidates' first 16 bytes at once (independent loads); a
        // slot may already hold a later position of this round (no barrier
        // between reads and inserts): only earlier positions within 32 KiB
        // are candidates
        uint32_t L[kMine], D[kMine];
  #pragma unroll
        for (uint32_t k = 0; k < kMine; k++) {
          const uint32_t e = (cs[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
          const uint32_t q = e - 1u;
          const bool ok = e != 0u && q < w && w - q <= kWindow;
          uint32_t wq[4];
          win16(hist, data, hw, (ok ? q : 0u) + sh, wq);
          L[k] = ok ? eq16(cur, wq) : 0u;
          D[k] = w - q;
        }
  #pragma unroll
        for (uint32_t k = 0; k < kMine; k++) {
          uint32_t Lk = L[k];
          if (Lk == 16u && lim > 16u)  // rare: extend past 16 bytes
            Lk = 16u + match_len(hist, data, hw, sh, p + 16u, w - D[k] + 16u, lim - 16u);
          Lk = min(Lk, lim);
          // a 4-byte match farther than kFar4 costs more bits than its four
          // literals (length and distance codes with >= 9 extra bits)
          if (Lk >= 4u && !(Lk == 4u && D[k] > kFar4) && (Lk > bl || (Lk == bl && D[k] < best))) {
            bl = Lk;
            best = D[k];
          }
        }
      }
      if (r + 1u < kSeg / kRound) seg16(data, p + kRound + sh, curn);
      if constexpr (kPair == 2u) {
        // the partner lane's result by a DPP quad permutation [1,0,3,2] (no LDS trip)
        const uint32_t obl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)bl, 0xB1, 0xF, 0xF, false);
        const uint32_t obest = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)best, 0xB1, 0xF, 0xF, false);
        if (obl > bl || (obl == bl && obest < best)) {
          bl = obl;
          best = obest;
        }
      }
      if (part == 0u) {
        cdg[p] = (uint16_t)best;
        lg[p] = (uint8_t)(bl ? bl - 3u : 0u);
      }
      __syncthreads();
    }
    // the distances back into LDS over the table (8 positions = 4 words per
    // load, never split by a pad dword); the barrier above ordered the
    // slot's stores before these loads within the workgroup
    static_assert((kSub / 2) % 4u == 0u, "pad groups hold whole 4-word runs");
    for (uint32_t k = t; k < kSeg / 8u; k += kThreads) {
      const uint4 v = reinterpret_cast<const uint4*>(cdg)[k];
      const uint32_t wd = 4u * k, ph = wd + (wd >> kCdShift);
      tab[ph] = v.x;
      tab[ph + 1u] = v.y;
      tab[ph + 2u] = v.z;
      tab[ph + 3u] = v.w;
    }
    // the lengths into the history's LDS (no longer read: the parse takes
    // lengths from here, literals from the segment's words)
    static_assert(kSeg <= 4u * kHistWords, "the lengths fit the history's LDS");
    for (uint32_t k = t; k < kSeg / 16u; k += kThreads) {
      const uint4 v = reinterpret_cast<const uint4*>(lg)[k];
      const uint32_t w0 = 4u * k, sw = (w0 >> 4) & 15u;
      hist[w0 ^ sw] = v.x;
      hist[(w0 + 1u) ^ sw] = v.y;
      hist[(w0 + 2u) ^ sw] = v.z;
      hist[(w0 + 3u) ^ sw] = v.w;
    }
    __syncthreads();

    K7P(3);
    // 2. the parse: dry passes hand each thread's end on as the next
    //    thread's start until no start moves, then the recording pass
    const uint32_t r0 = min(t * kSub, n), rend = min(r0 + kSub, n);
    uint32_t extra, my_s = r0;
    uint64_t mask = 0ull;
    uint32_t e_t = parse<false>(data, l8, cd, hll, hd, sh, n, my_s, rend, 0u, fbits, extra, &mask, r0);
    bool converged = false;  // workgroup-uniform
    for (uint32_t it = 0; it < kParseRounds; it++) {
      if (t + 1u < kThreads) starts[t + 1u] = e_t;
      __syncthreads();
      const uint32_t ns = t ? starts[t] : 0u;
      const bool moved = ns != my_s;
      if (!__syncthreads_or(moved)) {
        converged = true;
        break;
      }
      if (moved) {
        my_s = ns;
        e_t = parse<false>(data, l8, cd, hll, hd, sh, n, my_s, rend, 0u, fbits, extra, &mask, r0);
      }
    }
    K7P(4);
    if (!converged) {
      // The hand-off did not settle (all-zero data cycles with period 4):
      // starts[t] is thread t-1's latest end and starts[t+1] thread t's, and a
      // re-parsed thread t-1 may now end past thread t's end.  The recording
      // ranges [starts[t], starts[t+1]) must tile [0, n) exactly, so they are
      // made ascending by a running maximum (an empty range records nothing;
      // the final parse clips its matches to the range end).
      if (t == 0u) {
        uint32_t m = 0u;
        for (uint32_t k = 1u; k < kThreads; k++) {
          m = max(m, starts[k]);
          starts[k] = m;
        }
      }
      __syncthreads();
    }
    p_s = t ? starts[t] : 0u;
    p_e = t + 1u < kThreads ? starts[t + 1u] : n;
    // converged: the last dry pass's tokens end exactly at the next start
    if (converged && p_s == my_s && e_t == p_e)
      record_tokens(data, cd, hll, hd, sh, r0, mask, e_t, fbits, extra);
    else
      (void)parse<true>(data, l8, cd, hll, hd, sh, n, p_s, rend, p_e, fbits, extra);
    K7P(5);
    // the tokens, each thread's range and fixed-code bits, and the symbol
    // counts go to the slot for K7h (the distances and lengths there are
    // consumed); the EOB is not counted here
    const uint32_t xs[2] = {fbits, extra};
    uint32_t ts[2];
    (void)wg_sums<2>(xs, wsum4, ts);  // its barriers also order the counts' atomics
    for (uint32_t k = t; k < kCdPhys / 2u; k += kThreads) slot[k] = tab[k];
    slot[kSlotThr + t] = p_s;
    slot[kSlotThr + kThreads + t] = p_e;
    slot[kSlotThr + 2u * kThreads + t] = fbits;
    uint32_t* const rec = slot + kSlotRec;
    if (t < 320u) rec[t] = t < 286u ? (t == 256u ? 0u : hll[t]) : (t >= 288u && t < 318u ? hd[t - 288u] : 0u);
    if (t == 0u) {
      rec[320] = ts[0];
      rec[321] = ts[1];
    }
  }
}


// K7h: codes one parsed segment from K7a's hand-off in its slot.  The parsed
// segments of a group (kGroup consecutive segments of one block, none stored
// by K7e) share one dynamic code built from their summed counts: the first
// member's bits start with the header, the last member's end with the end of
// block and the sync flush, and member m's bits continue member m-1's at bit
// S_m = header + the bits of members 0..m-1 (each member's bit count follows
// from its counts and the code's lengths).  Every member builds the same code
// from the same counts, so the decision and every offset agree across the
// group's workgroups with no communication between them.  A member's image
// starts at bit S_m mod 8 of the byte K7b ORs it into (S_m / 8 of the piece).
// The group shares only if its piece is smaller than the sum of its members'
// fixed-or-stored sizes; otherwise each member is coded
// alone (dynamic, fixed or stored, whichever is smallest; rounds 1-4).
extern "C" __global__ __launch_bounds__(hbxz::kThreads) void hbx_k7_deflate_code(const hbxz::ZBlock* __restrict__ blocks,
                                                                                uint32_t nb, uint32_t nseg,
                                                                                hbxz::SegInfo* __restrict__ info,
                                                                                uint32_t* __restrict__ scratch) {
  using namespace hbxz;
  __shared__ __attribute__((aligned(16))) uint32_t cdw[kCdPhys / 2u];  // the tokens
  const uint16_t* const cd = reinterpret_cast<const uint16_t*>(cdw);
  __shared__ __attribute__((aligned(16))) uint32_t win[kImgWords];  // Huffman scratch, then the image
  __shared__ uint32_t mrec[kGroup][kRecWords];
  __shared__ uint32_t wsum[kWaves];
  __shared__ uint32_t wsum4[4 * kWaves];
  __shared__ uint32_t hll[288], hd[32], llc[288], dcc[32], rle[320], clf[19], clc[19], zpar[8], zctl[8];
  __shared__ uint32_t gpar[3 * kGroup + 2];
  __shared__ __attribute__((aligned(4))) uint8_t zl[320];
  __shared__ uint8_t cll[20];
  __shared__ unsigned long long rmask[5];  // code-length run starts (header RLE)
  static_assert(6464u <= kImgWords, "the Huffman scratch fits the image's LDS");
  static_assert(kGroup <= 8u, "member bit sums in zctl");
  const uint32_t g = blockIdx.x;
  if (g >= nseg) return;
  const SegInfo si0 = info[g];
  if (si0.mode == kModeSrcStored) return;
  K7P(6);
  const ZBlock bk = blocks[zblock_of(blocks, nb, g)];
  const uint32_t s = g - bk.seg0;
  const uint32_t n = (uint32_t)min((uint64_t)kSeg, bk.len - (uint64_t)s * kSeg);
  const uint32_t t = threadIdx.x;
  const uint32_t gs = s - s % kGroup, gn = min(kGroup, bk.nseg - gs), my = s - gs;
  uint32_t* const slot = scratch + (uint64_t)g * (kSlot / 4u);
  for (uint32_t k = t; k < kCdPhys / 2u; k += kThreads) cdw[k] = slot[k];
  const uint32_t p_s = slot[kSlotThr + t], p_e = slot[kSlotThr + kThreads + t];
  const uint32_t fbits = slot[kSlotThr + 2u * kThreads + t];
  // a member's mode is K7e's (parse or stored) or, once its own K7h has
  // coded it, 1/2/4/5/kModeOwnStored: never kModeSrcStored, so "not stored by
  // K7e" reads the same before and after a sibling's write (kModeOwnStored)
  const bool live = t >= gn || info[bk.seg0 + gs + t].mode != kModeSrcStored;
  const bool grp = __syncthreads_and(live) && gn >= 2u;
  const uint32_t own = grp ? my : 0u;
  for (uint32_t m = 0; m < kGroup; m++) {
    if (!(grp ? m < gn : m == 0u)) continue;
    const uint32_t* rec = scratch + (uint64_t)(grp ? g - my + m : g) * (kSlot / 4u) + kSlotRec;
    for (uint32_t k = t; k < kRecWords; k += kThreads) mrec[m][k] = rec[k];
  }
  __syncthreads();
  uint32_t fincl, ftot;
  fincl = wg_incl_sum(fbits, wsum, ftot);
  const uint32_t stored_bytes = 5u + n;
  const uint32_t fixed_bytes = ((3u + ftot + 7u + 3u + 7u) >> 3) + 4u;  // header, tokens, EOB, sync flush
  uint32_t hoff = 0u;  // dynamic header: bit offset of run-length symbol t among them
  uint32_t mode = 0u, nbytes = stored_bytes, ibase = 0u;
  bool shared = false;
  #pragma nounroll
  for (uint32_t pass = grp ? 0u : 1u; pass < 2u; pass++) {
    const bool G = pass == 0u;  // the group's code, else this segment's own
    if (t < 320u) {
      uint32_t c = 0u;
      if (G) {
        for (uint32_t m = 0; m < gn; m++) c += mrec[m][t];
      } else {
        c = mrec[own][t];
      }
      if (t == 256u) c = 1u;  // the EOB, once
      if (t < 288u) hll[t] = c; else hd[t - 288u] = c;
    }
    __syncthreads();
    uint32_t etot = 0u;
    for (uint32_t m = 0; m < (G ? gn : 1u); m++) etot += mrec[G ? m : own][321];
    // the entropy estimate of a dynamic code (alone: build one only if it can win)
    const uint32_t f_t = t < 286u ? hll[t] : (t >= 288u && t < 318u ? hd[t - 288u] : 0u);
    uint32_t ntok, ndist;
    {
      const uint32_t xs[2] = {t < 286u ? f_t : 0u, t >= 288u ? f_t : 0u};
      uint32_t ts[2];
      (void)wg_sums<2>(xs, wsum4, ts);
      ntok = ts[0];
      ndist = ts[1];
    }
    K7P(12);
    const float nn = t < 286u ? (float)ntok : (float)max(ndist, 1u);
    const uint32_t h_t = f_t ? (uint32_t)((float)f_t * (__log2f(nn) - __log2f((float)f_t))) : 0u;
    uint32_t htot;
    (void)wg_incl_sum(h_t, wsum, htot);
    K7P(13);
    const uint32_t best_other = min(fixed_bytes, stored_bytes) * 8u;
    const bool try_dyn = G || htot + etot + 600u < best_other;
    if (try_dyn) {
      // scratch in the window (idle since the recording pass)
      uint32_t* keys = win;                                      // 512 litlen keys, sorted
      uint32_t* keysd = win + 512;                               // 32 distance keys, sorted
      uint32_t* hw = win + 576;                                  // weights: litlen 572, distance 60 at +576
      uint32_t* npar = win + 1792;                               // tree parents, distance nodes at +576
      uint32_t* nanc = win + 2816;                               // pointer-jumping ancestors
      uint32_t* ndep = win + 3840;                               // depths
      uint32_t* blc = win + 4864;                                // 2 x 16 length counts
      for (uint32_t k = t; k < 512u; k += kThreads) keys[k] = (k < 286u && hll[k]) ? (hll[k] << 9) | k : 0xFFFFFFFFu;
      // the sort's compare source: litlen keys at 0..287, distance keys at 288..319
      uint32_t* ksrc = win + 6144;
      for (uint32_t k = t; k < 320u; k += kThreads)
        ksrc[k] = k < 286u   ? (hll[k] ? (hll[k] << 9) | k : 0xFFFFFFFFu)
                : k < 288u   ? 0xFFFFFFFFu
                : k < 318u   ? (hd[k - 288u] ? (hd[k - 288u] << 9) | (k - 288u) : 0xFFFFFFFFu)
                             : 0xFFFFFFFFu;
      for (uint32_t k = t; k < 320u; k += kThreads) zl[k] = 0u;
      if (t < 32u) blc[t] = 0u;
      if (t < 19u) clf[t] = 0u;
      if (t < 8u) zctl[t] = 0u;
      __syncthreads();
      K7P(14);
      // rank sorts, ascending (keys are unique: the symbol is in the low
      // bits): thread t < 286 places litlen symbol t, thread 288 + k distance
      // symbol k.  (A one-wave bitonic sort of 512 keys took ~25 % of the
      // segment's code construction; one compare per LDS read or readlane
      // 32 k cycles, four per read 9 k.)
      {
        // every thread compares its key with all of them, four per LDS
        // broadcast read (ksrc: the keys of symbol order, absent = ~0u)
        const uint4* k4 = reinterpret_cast<const uint4*>(ksrc);
        if (t < 286u && hll[t] != 0u) {
          const uint32_t key = (hll[t] << 9) | t;
          uint32_t r = 0u;
  #pragma unroll 8
          for (uint32_t q = 0; q < 288u / 4u; q++) {
            const uint4 v = k4[q];
            r += (v.x < key) + (v.y < key) + (v.z < key) + (v.w < key);
          }
          keys[r] = key;
        } else if (t >= 288u && t < 318u) {
          const uint32_t k = t - 288u;
          if (hd[k]) {
            const uint32_t key = (hd[k] << 9) | k;
            uint32_t r = 0u;
  #pragma unroll
            for (uint32_t q = 288u / 4u; q < 320u / 4u; q++) {
              const uint4 v = k4[q];
              r += (v.x < key) + (v.y < key) + (v.z < key) + (v.w < key);
            }
            keysd[r] = key;
          }
        }
      }
      const uint32_t ml = (uint32_t)__syncthreads_count(t < 286u && hll[t] != 0u);  // >= 1 (EOB)
      K7P(8);
      const uint32_t md = (uint32_t)__syncthreads_count(t < 30u && hd[t] != 0u);
      // Huffman trees of both codes at once: the serial merges on two waves,
      // then depths by pointer jumping over every node; halve and rebuild a
      // code whose longest length exceeds 15.
      bool need_l = ml >= 2u, need_d = md >= 2u;
      for (uint32_t shift = 0; need_l || need_d; shift++) {
        if (t == 0u && need_l) huff_merge(keys, ml, shift, hw, npar, 0u);
        if (t == 64u && need_d) huff_merge(keysd, md, shift, hw + 576, npar + 576, 576u);
        if (t < 2u) zctl[t] = 0u;
        __syncthreads();
        // nodes 0 .. 576 + 59: x1 only while kThreads < 1024 (with 1024 threads
        // x1 = x0 + 1024 would run past the scratch)
        static_assert(kThreads == 512u || kThreads == 1024u, "node cover");
        uint32_t x0 = t, x1 = kThreads < 1024u ? t + kThreads : t, a0, a1, d0, d1;
        auto init = [&](uint32_t x, uint32_t& a, uint32_t& d) {
          const bool dist = x >= 576u;
          const uint32_t m = dist ? md : ml, root = (dist ? 576u : 0u) + 2u * m - 2u;
          const bool live = m >= 2u && x <= root && x >= (dist ? 576u : 0u);
          a = live && x != root ? npar[x] : x;
          d = live && x != root ? 1u : 0u;
        };
        init(x0, a0, d0);
        init(x1, a1, d1);
        nanc[x0] = a0;
        nanc[x1] = a1;
        ndep[x0] = d0;
        ndep[x1] = d1;
        __syncthreads();
        for (int r = 0; r < 10; r++) {  // depth <= 571 < 2^10
          const uint32_t e0 = ndep[a0], e1 = ndep[a1], b0 = nanc[a0], b1 = nanc[a1];
          __syncthreads();
          d0 += e0;
          d1 += e1;
          a0 = b0;
          a1 = b1;
          ndep[x0] = d0;
          ndep[x1] = d1;
          nanc[x0] = a0;
          nanc[x1] = a1;
          __syncthreads();
        }
        if (x0 < ml) atomicMax(&zctl[0], d0);
        if (x0 >= 576u && x0 < 576u + md) atomicMax(&zctl[1], d0);
        if (x1 >= 576u && x1 < 576u + md) atomicMax(&zctl[1], d1);
        __syncthreads();
        need_l = need_l && zctl[0] > 15u;
        need_d = need_d && zctl[1] > 15u;
        __syncthreads();
      }
      K7P(9);
      // code lengths (one distance symbol gets a second: RFC 1951 §3.2.7)
      if (t < ml) zl[keys[t] & 511u] = ml >= 2u ? (uint8_t)ndep[t] : 1u;
      if (md >= 2u && t < md) zl[288u + (keysd[t] & 511u)] = (uint8_t)ndep[576u + t];
      if (md == 0u && t < 2u) zl[288u + t] = 1u;
      if (md == 1u && t < 2u) {
        const uint32_t x = keysd[0] & 511u;
        zl[288u + (t ? (x ? 0u : 1u) : x)] = 1u;
      }
      __syncthreads();
      // HLIT, HDIST, per-length counts
      const uint32_t zt = t < 286u ? zl[t] : (t >= 288u && t < 318u ? zl[t] : 0u);
      if (zt) atomicAdd(&blc[(t >= 288u ? 16u : 0u) + zt], 1u);
      if (zt && t >= 257u && t < 286u) atomicMax(&zctl[2], t + 1u);
      if (zt && t >= 288u) atomicMax(&zctl[3], t - 288u + 1u);
      __syncthreads();
      const uint32_t hlit = max(zctl[2], 257u), hdist = max(zctl[3], 1u);
      // canonical codes (RFC 1951 §3.2.2): first code of the length + the rank
      // among the symbols of that length before this one
      if (zt) {
        const uint32_t cb = t >= 288u ? 16u : 0u, s0 = t >= 288u ? 288u : 0u;
        uint32_t code = 0u;
        for (uint32_t b = 1; b <= zt; b++) code = (code + (b > 1u ? blc[cb + b - 1u] : 0u)) << 1;
        const uint32_t* zw = reinterpret_cast<const uint32_t*>(zl);
        const uint32_t pat = zt * 0x01010101u;
        uint32_t rank = 0u;
        for (uint32_t q = s0; q < t; q += 4u) {
          uint32_t v = zw[q >> 2] ^ pat;
          if (t - q < 4u) v |= 0xFFFFFFFFu << (8u * (t - q));  // bytes at or past t never count
          const uint32_t y = ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
          rank += __builtin_popcount(y);
        }
        const uint32_t c = rev(code + rank, zt) | (zt << 16);
        if (t >= 288u) dcc[t - 288u] = c; else llc[t] = c;
      } else if (t < 286u) {
        llc[t] = 0u;
      } else if (t >= 288u && t < 318u) {
        dcc[t - 288u] = 0u;
      }
      K7P(10);
      // code-length sequence, run-length coded (16/17/18): one thread per run
      const uint32_t nl = hlit + hdist;
      auto zv = [&](uint32_t i) -> uint32_t { return i < hlit ? zl[i] : zl[288u + i - hlit]; };
      uint32_t cur = 0u, run = 0u, cnt = 0u;
      // run starts as one bit mask per wave (nl <= 316: waves 0..4); a run
      // ends at the next start
      const bool rstart = t < nl && (t == 0u || zv(t - 1u) != zv(t));
      const uint64_t bm = __builtin_amdgcn_ballot_w64(rstart);
      if ((t & 63u) == 0u && t < 320u) rmask[t >> 6] = bm;
      __syncthreads();
      if (rstart) {
        cur = zv(t);
        const uint32_t wv = t >> 6, b = t & 63u;
        uint64_t m = b < 63u ? rmask[wv] & (~0ull << (b + 1u)) : 0ull;
        uint32_t w2 = wv;
        while (m == 0ull && ++w2 < 5u) m = rmask[w2];
        const uint32_t nx = m ? min(nl, 64u * w2 + (uint32_t)__builtin_ctzll(m)) : nl;
        run = nx - t;
        cnt = rle_runs<false>(cur, run, nullptr, nullptr);
      }
      uint32_t nr;
      const uint32_t at = wg_incl_sum(cnt, wsum, nr) - cnt;
      if (cnt) rle_runs<true>(cur, run, rle + at, clf);
      __syncthreads();
      if (t < 64u) {  // the code-length code: one wave
        const uint32_t hcl = cl_code(t < 19u ? clf[t] : 0u, cll, clc);
        if (t == 0u) zctl[4] = hcl;
      }
      __syncthreads();
      const uint32_t hclen = zctl[4];
      K7P(11);
      uint32_t hcost = 0u, tcost = 0u, hb_body, tok_body;
      if (t < nr) {
        const uint32_t sy = rle[t] & 31u;
        hcost = (clc[sy] >> 16) + (sy == 16u ? 2u : sy == 17u ? 3u : sy == 18u ? 7u : 0u);
      }
      if (t < 286u) tcost = hll[t] * zl[t];  // EOB included (hll[256] = 1)
      else if (t >= 288u && t < 318u) tcost = hd[t - 288u] * zl[t];
      hoff = wg_incl_sum(hcost, wsum, hb_body) - hcost;
      (void)wg_incl_sum(tcost, wsum, tok_body);
      if (t == 0) {
        const uint32_t hb = 3u + 5u + 5u + 4u + 3u * hclen + hb_body;
        const uint32_t dyn_bytes = ((hb + etot + tok_body + 3u + 7u) >> 3) + 4u;
        zpar[0] = dyn_bytes < min(fixed_bytes, stored_bytes) ? 2u : 0u;
        zpar[1] = hb;
        zpar[2] = dyn_bytes;
        zpar[3] = hlit | (hdist << 16);
        zpar[4] = hclen | (nr << 16);
      }
      __syncthreads();
    } else if (t == 0) {
      zpar[0] = 0u;
    }
    __syncthreads();
    if (G) {
      // each member's bits under the group's code, its place in the piece
      if (t < kGroup) zctl[t] = 0u;
      __syncthreads();
      if (t < 320u && zl[t])
        for (uint32_t m = 0; m < gn; m++) atomicAdd(&zctl[m], mrec[m][t] * zl[t]);
      __syncthreads();
      if (t < gn) atomicAdd(&zctl[t], mrec[t][321]);  // + its extra bits
      __syncthreads();
      if (t == 0u) {
        const uint32_t hb = zpar[1], eob = llc[256] >> 16;
        uint32_t S = hb, alone = 0u, ok = 1u, total = 0u;
        for (uint32_t m = 0; m < gn; m++) {
          const uint32_t T = zctl[m];
          const uint32_t o0 = m ? (S & 7u) : hb;  // where its first token goes in its image
          const uint32_t B = m ? (S >> 3) : 0u;
          const uint32_t end = o0 + T;
          const uint32_t il = m + 1u == gn ? ((end + eob + 3u + 7u) >> 3) + 4u : (end + 7u) >> 3;
          if (il + 8u > 4u * kImgWords) ok = 0u;
          gpar[3 * m] = B;
          gpar[3 * m + 1] = il;
          gpar[3 * m + 2] = o0;
          S += T;
          total = B + il;
          const uint32_t nm = (uint32_t)min((uint64_t)kSeg, bk.len - (uint64_t)(gs + m) * kSeg);
          const uint32_t fm = ((3u + mrec[m][320] + 7u + 3u + 7u) >> 3) + 4u;
          alone += min(5u + nm, fm);
        }
        gpar[3 * kGroup] = ok && total < alone ? 1u : 0u;
        gpar[3 * kGroup + 1] = total;
      }
      __syncthreads();
      shared = gpar[3 * kGroup] != 0u;
      if (shared) {
        mode = 2u;
        ibase = gpar[3 * my + 2];
        nbytes = gpar[3 * my + 1];
        break;
      }
      continue;  // code alone
    }
    mode = zpar[0];  // 2 dynamic, 0 not (then fixed or stored)
    if (mode == 0u && fixed_bytes < stored_bytes) mode = 1u;
    ibase = mode == 2u ? zpar[1] : 3u;
  }
  if (mode == 1u) {  // fixed code tables
    for (uint32_t k = t; k < 288u; k += kThreads)
      llc[k] = k < 144u ? rev(0x30u + k, 8u) | (8u << 16)
             : k < 256u ? rev(0x190u + k - 144u, 9u) | (9u << 16)
             : k < 280u ? rev(k - 256u, 7u) | (7u << 16)
                        : rev(0xC0u + k - 280u, 8u) | (8u << 16);
    for (uint32_t k = t; k < 32u; k += kThreads) dcc[k] = rev(k, 5u) | (5u << 16);
  }
  K7P(7);
  uint32_t* img = win;  // the Huffman scratch is idle now
  if (mode != 0u) {
    __syncthreads();
    for (uint32_t k = t; k < kImgWords; k += kThreads) img[k] = 0u;
    __syncthreads();
    // this thread's tokens at its prefix offset after the block header (or,
    // in a group, after the bits before it in its first byte)
    uint32_t mine = fbits, incl = fincl, tot = ftot;
    if (mode == 2u) {
      mine = walk_tokens<false>(cd, llc, dcc, nullptr, p_s, p_e, 0u);
      incl = wg_incl_sum(mine, wsum, tot);
    }
    const bool head = !shared || my == 0u, last = !shared || my + 1u == gn;
    if (mode == 1u) {
      if (t == 0) {
        uint32_t o = 0u;
        emit_bits(img, o, 2u, 3u);  // BFINAL 0, BTYPE 01
      }
    } else if (head) {
      // the dynamic block header, one field per thread at its bit offset
      const uint32_t hlit = zpar[3] & 0xFFFFu, hdist = zpar[3] >> 16;
      const uint32_t hclen = zpar[4] & 0xFFFFu, nr = zpar[4] >> 16;
      if (t == 0) {
        uint32_t o = 0u;
        emit_bits(img, o, 4u, 3u);  // BFINAL 0, BTYPE 10
        emit_bits(img, o, hlit - 257u, 5u);
        emit_bits(img, o, hdist - 1u, 5u);
        emit_bits(img, o, hclen - 4u, 4u);
      }
      if (t < hclen) {  // code-length code lengths, 3 bits each, in kClOrder
        uint32_t o = 17u + 3u * t;
        emit_bits(img, o, cll[kClOrder[t]], 3u);
      }
      if (t < nr) {  // run-length coded code lengths (hoff: the prefix of their bits)
        uint32_t o = 17u + 3u * hclen + hoff;
        const uint32_t sy = rle[t] & 31u, e = clc[sy];
        emit_bits(img, o, e & 0xFFFFu, e >> 16);
        if (sy >= 16u) emit_bits(img, o, rle[t] >> 8, sy == 16u ? 2u : sy == 17u ? 3u : 7u);
      }
    }
    walk_tokens<true>(cd, llc, dcc, img, p_s, p_e, ibase + incl - mine);
    __syncthreads();
    if (t == 0) {
      uint32_t o = ibase + tot, e = (o + 7u) >> 3;
      if (last) {
        emit_bits(img, o, llc[256] & 0xFFFFu, llc[256] >> 16);  // end of block
        e = (o + 3u + 7u) >> 3;                                 // + the empty stored block's 3 header bits
        uint8_t* ob = reinterpret_cast<uint8_t*>(img);
        ob[e] = 0x00;
        ob[e + 1] = 0x00;
        ob[e + 2] = 0xFF;
        ob[e + 3] = 0xFF;
        e += 4u;
      }
      zpar[5] = e;
    }
    __syncthreads();
    nbytes = zpar[5];  // in a group: equal to gpar's il (the walk and the counts agree)
  } else {
    mode = kModeOwnStored;  // stored: K7b copies the bytes from the source
  }
  if (mode != kModeOwnStored)
    for (uint32_t k = t; k < (nbytes + 3u) / 4u; k += kThreads) slot[k] = img[k];
  if (t == 0) {
    SegInfo si = si0;
    if (shared) {
      slot[kSlotMeta] = gpar[3 * my];
      slot[kSlotMeta + 1] = nbytes;
      slot[kSlotMeta + 2] = gn;
      si.mode = my == 0u ? kModeGroupHead : kModeGroupMember;
      si.bytes = my == 0u ? gpar[3 * kGroup + 1] : 0u;
    } else {
      si.mode = mode;
      si.bytes = nbytes;
    }
    info[g] = si;
  }
  K7P(15);
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
                                                                        const uint64_t* __restrict__ seg_off,
                                                                        const hbxz::ZBlock* __restrict__ blocks,
                                                                        uint32_t nb) {
  using namespace hbxz;
  __shared__ uint32_t img[kImgWords + 2];
  const uint32_t g = blockIdx.x;
  if (g >= nseg) return;
  const uint32_t t = threadIdx.x;
  const SegInfo si = info[g];
  const uint32_t nbytes = si.bytes;
  if (si.mode == kModeGroupMember) return;  // written with its group's head
  if (si.mode == kModeSrcStored || si.mode == kModeOwnStored) {  // 00 | LEN | ~LEN | the segment's bytes, straight from the source
    const ZBlock bk = blocks[zblock_of(blocks, nb, g)];
    const uint32_t n = nbytes - 5u;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(bk.src) + (uint64_t)(g - bk.seg0) * kSeg;
    uint8_t* D = reinterpret_cast<uint8_t*>(seg_off[g]);
    const uint8_t hdr[5] = {0u, (uint8_t)n, (uint8_t)(n >> 8), (uint8_t)~n, (uint8_t)(~n >> 8)};
    auto byte_at = [&](uint32_t q) -> uint32_t { return q < 5u ? hdr[q] : src[q - 5u]; };
    const uint32_t lead = (uint32_t)((4u - (reinterpret_cast<uint64_t>(D) & 3u)) & 3u);
    const uint32_t head = min(lead, nbytes);
    if (t < head) D[t] = (uint8_t)byte_at(t);
    const uint32_t nw = (nbytes - head) >> 2;
    uint32_t* Dw = reinterpret_cast<uint32_t*>(D + head);
    for (uint32_t k = t; k < nw; k += kWThreads) {
      const uint32_t q = head + 4u * k;
      uint32_t w;
      if (q >= 5u) {  // four source bytes at any alignment (the hardware splits the load)
        w = *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(
            reinterpret_cast<uintptr_t>(src + (q - 5u)));
      } else {
        w = byte_at(q) | (byte_at(q + 1u) << 8) | (byte_at(q + 2u) << 16) | (byte_at(q + 3u) << 24);
      }
      Dw[k] = w;
    }
    const uint32_t done = head + 4u * nw;
    if (t < nbytes - done) D[done + t] = (uint8_t)byte_at(done + t);
    return;
  }
  const uint32_t* slot = scratch + (uint64_t)g * (kSlot / 4u);
  if (si.mode == kModeGroupHead) {
    // the group's piece, straight from the members' images: member m's
    // image covers piece bytes [B_m, B_m + il_m), and where two members meet
    // a byte holds bits of both (OR).  No LDS: this path would otherwise set
    // K7b's LDS, and with it the occupancy of the stored-segment copies.
    const uint32_t gn = slot[kSlotMeta + 2];
    uint32_t Bm[kGroup], Lm[kGroup];
    const uint8_t* Mb[kGroup];
  #pragma unroll
    for (uint32_t m = 0; m < kGroup; m++) {
      const uint32_t* ms = scratch + (uint64_t)(g + min(m, gn - 1u)) * (kSlot / 4u);
      Bm[m] = m < gn ? ms[kSlotMeta] : 0u;
      Lm[m] = m < gn ? ms[kSlotMeta + 1] : 0u;
      Mb[m] = reinterpret_cast<const uint8_t*>(ms);
    }
    auto piece4 = [&](uint32_t q) -> uint32_t {  // piece bytes q .. q + 3, little-endian
      uint32_t v = 0u;
  #pragma unroll
      for (uint32_t m = 0; m < kGroup; m++) {
        if (q + 4u <= Bm[m] || q >= Bm[m] + Lm[m]) continue;  // also every m >= gn (Lm = 0)
        const int32_t r = (int32_t)q - (int32_t)Bm[m];
        if (r >= 0 && (uint32_t)r + 4u <= Lm[m]) {  // four image bytes at any alignment
          v |= *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(
              reinterpret_cast<uintptr_t>(Mb[m] + r));
        } else {
          for (int32_t j = 0; j < 4; j++)
            if (r + j >= 0 && (uint32_t)(r + j) < Lm[m]) v |= (uint32_t)Mb[m][r + j] << (8 * j);
        }
      }
      return v;
    };
    uint8_t* D = reinterpret_cast<uint8_t*>(seg_off[g]);
    const uint32_t lead = (uint32_t)((4u - (reinterpret_cast<uint64_t>(D) & 3u)) & 3u);
    const uint32_t head = min(lead, nbytes);
    if (t < head) D[t] = (uint8_t)piece4(t);
    const uint32_t nw = (nbytes - head) >> 2;
    uint32_t* Dw = reinterpret_cast<uint32_t*>(D + head);
    for (uint32_t k = t; k < nw; k += kWThreads) Dw[k] = piece4(head + 4u * k);
    const uint32_t done = head + 4u * nw;
    if (t < nbytes - done) D[done + t] = (uint8_t)piece4(done + t);
    return;
  }
  for (uint32_t k = t; k < kImgWords + 2u; k += kWThreads) img[k] = k < (nbytes + 3u) / 4u ? slot[k] : 0u;
  __syncthreads();
  // image [0, nbytes) -> the stream at byte address D
  uint8_t* D = reinterpret_cast<uint8_t*>(seg_off[g]);
  const uint32_t lead = (uint32_t)((4u - (reinterpret_cast<uint64_t>(D) & 3u)) & 3u);
  const uint32_t head = min(lead, nbytes);
  const uint8_t* ob = reinterpret_cast<const uint8_t*>(img);
  if (t < head) D[t] = ob[t];
  const uint32_t nw = (nbytes - head) >> 2;
  uint32_t* Dw = reinterpret_cast<uint32_t*>(D + head);
  for (uint32_t k = t; k < nw; k += kWThreads) Dw[k] = lds4(img, head + 4u * k);
  const uint32_t done = head + 4u * nw;
  if (t < nbytes - done) D[done + t] = ob[done + t];
}

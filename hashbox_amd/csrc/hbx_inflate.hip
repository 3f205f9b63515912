// hbx_inflate.hip — zlib inflate on gfx950, one lane per stream (the read
// side of SURVEY §8f2/§8f4).
//
// Reference: HashboxBlock.UncompressData / zlibUncompress (pkg/core/
// block.go:113-131, 186-201) before VerifyBlock hashes a stored block
// (block.go:152-174): restore (hashback/restore.go:52, 256), the server's
// write check (server/server.go:182), verify -content (pkg/storagedb/
// integrity.go:117, 282).  The streams come from Go's compress/zlib (or from
// K7), so this is a general RFC 1950/1951 decoder: stored, fixed and dynamic
// blocks, any window distance.
//
// A stream is serial, so a lane decodes one stream (64 per wave; the host
// sorts streams longest first).  Huffman decoding is canonical (RFC 1951
// §3.2.2): the codes of length l are the consecutive values [first[l],
// limit[l]), so a decoder peeks 15 bits, bit-reverses them (codes are sent
// most significant bit first) and takes the shortest l whose l-bit prefix is
// below limit[l]; the symbol is sym[prefix + base[l]].  The tables live in LDS
// per lane.  Every read and write is bounds-checked: a corrupt stream sets its
// status and stops, it never touches memory outside its input and output.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hbxi {

constexpr uint32_t kLanes = 64;
constexpr uint32_t kLenSyms = 288, kDistSyms = 32;

// status codes (out_status)
constexpr uint32_t kOk = 0, kErrHeader = 1, kErrInput = 2, kErrOutput = 3, kErrCode = 4, kErrDist = 5,
                   kErrStored = 6;

// One canonical code: limit[l] = first code of length l + number of codes
// of length l (l-bit code space); base[l] = index in sym of the first symbol
// of length l minus the first code of length l.
struct Code {
  uint16_t limit[16];
  int16_t base[16];
};

struct LaneTables {
  Code lc, dc;
  uint16_t next[16];  // placement cursors while a table is built
  uint16_t lsym[kLenSyms];
  uint16_t dsym[kDistSyms];
  uint8_t lens[320];  // code lengths while a dynamic table is built
  uint8_t dlens[32];
};

__device__ const uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                          31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__device__ const uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct Bits {
  const uint8_t* start;
  const uint8_t* p;  // next byte to load (may run past `end`: zeros are loaded)
  const uint8_t* end;
  uint64_t buf;
  uint32_t n;  // bits in buf
  __device__ __forceinline__ void fill() {
    while (n <= 56u) {
      const uint32_t b = p < end ? (uint32_t)*p : 0u;
      p++;
      buf |= (uint64_t)b << n;
      n += 8u;
    }
  }
  // more bits consumed than the input holds (the look-ahead alone is fine)
  __device__ __forceinline__ bool overrun() const {
    return 8ull * (uint64_t)(p - start) - n > 8ull * (uint64_t)(end - start);
  }
  __device__ __forceinline__ uint32_t get(uint32_t k) {  // k <= 32
    if (n < k) fill();
    const uint32_t v = (uint32_t)(buf & ((1ull << k) - 1ull));
    buf >>= k;
    n -= k;
    return v;
  }
  __device__ __forceinline__ void align_byte() {
    const uint32_t k = n & 7u;
    buf >>= k;
    n -= k;
  }
};

// Next symbol of `c`, or -1 if the next 15 bits start no code of it.
__device__ __forceinline__ int decode(Bits& br, const Code& c, const uint16_t* sym) {
  if (br.n < 15u) br.fill();
  const uint32_t peek = __builtin_bitreverse32((uint32_t)br.buf) >> 17;  // first-sent bit on top
  for (uint32_t l = 1; l <= 15u; l++) {
    const uint32_t prefix = peek >> (15u - l);
    if (prefix < c.limit[l]) {
      br.buf >>= l;
      br.n -= l;
      return sym[(int)prefix + c.base[l]];
    }
  }
  return -1;
}

// The code of `n` symbols with code lengths `lens` (RFC 1951 §3.2.2 steps
// 1-3: count per length, first code per length, symbols in code order).
// Returns false when the lengths over-subscribe the code space; incomplete
// codes are accepted (a decoder meets a missing code only on corrupt input),
// and all-zero lengths give a code that decodes nothing.
__device__ __forceinline__ bool construct(Code& c, uint16_t* sym, uint16_t* next, const uint8_t* lens, int n) {
  uint16_t count[16];
  for (int l = 0; l < 16; l++) count[l] = 0;
  for (int s = 0; s < n; s++) count[lens[s]]++;
  count[0] = 0;
  int room = 1;  // unused codes of the current length (Kraft)
  uint32_t first = 0, start = 0;
  c.limit[0] = 0;
  c.base[0] = 0;
  for (int l = 1; l < 16; l++) {
    room = 2 * room - count[l];
    if (room < 0) return false;
    first = (first + count[l - 1]) << 1;
    c.limit[l] = (uint16_t)(first + count[l]);
    c.base[l] = (int16_t)((int)start - (int)first);
    next[l] = (uint16_t)start;
    start += count[l];
  }
  for (int s = 0; s < n; s++)
    if (lens[s]) sym[next[lens[s]]++] = (uint16_t)s;
  return true;
}

__device__ __forceinline__ uint32_t len_base(uint32_t s) { return kLenBase[s]; }  // s = symbol - 257, 0..28
__device__ __forceinline__ uint32_t len_extra(uint32_t s) {
  return s < 8u ? 0u : s == 28u ? 0u : (s - 4u) >> 2;
}
__device__ __forceinline__ uint32_t dist_base(uint32_t s) {  // 0..29
  return s < 4u ? s + 1u : ((2u + (s & 1u)) << ((s >> 1) - 1u)) + 1u;
}
__device__ __forceinline__ uint32_t dist_extra(uint32_t s) { return s < 4u ? 0u : (s >> 1) - 1u; }

// Non-overlapping copy, 16 independent byte loads in flight per step (the
// byte-at-a-time loop serialised on the possible aliasing of in and out).
__device__ __forceinline__ void copy_bytes(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, uint32_t n) {
  uint32_t j = 0;
  for (; j + 16u <= n; j += 16u) {
    uint8_t t[16];
#pragma unroll
    for (int q = 0; q < 16; q++) t[q] = src[j + q];
#pragma unroll
    for (int q = 0; q < 16; q++) dst[j + q] = t[q];
  }
  for (; j < n; j++) dst[j] = src[j];
}

// LZ77 copy of len bytes from dist back (dist <= bytes already written; the
// source may overlap the destination: then byte by byte)
__device__ __forceinline__ void copy_match(uint8_t* out, uint32_t dist, uint32_t len) {
  const uint8_t* src = out - dist;  // pointer arithmetic: never an unsigned wrap
  uint32_t j = 0;
  if (dist >= 16u) {
    for (; j + 16u <= len; j += 16u) {
      uint8_t t[16];
#pragma unroll
      for (int q = 0; q < 16; q++) t[q] = src[j + q];
#pragma unroll
      for (int q = 0; q < 16; q++) out[j + q] = t[q];
    }
  }
  for (; j < len; j++) out[j] = src[j];
}

}  // namespace hbxi

struct InflateDesc {
  uint64_t src;   // device address of the zlib stream
  uint64_t dst;   // device address of the output
  uint32_t len;   // stream bytes
  uint32_t cap;   // output capacity
};

// One lane per stream.  out_len[i] = inflated bytes, status[i] = 0 or an
// hbxi::kErr* code.
extern "C" __global__ __launch_bounds__(64) void hbx_k8_inflate(const InflateDesc* __restrict__ desc, uint32_t n,
                                                                 uint32_t* __restrict__ out_len,
                                                                 uint32_t* __restrict__ status) {
  using namespace hbxi;
  __shared__ LaneTables tabs[kLanes];
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  if (i >= n) return;
  LaneTables& T = tabs[threadIdx.x];
  const InflateDesc d = desc[i];
  const uint8_t* in = reinterpret_cast<const uint8_t*>(d.src);
  uint8_t* out = reinterpret_cast<uint8_t*>(d.dst);
  Bits br{in, in, in + d.len, 0ull, 0u};
  uint32_t o = 0u, st = kOk;
  // zlib header (RFC 1950 §2.2): deflate, 32 KiB window at most, check bits, no dictionary
  const uint32_t cmf = br.get(8), flg = br.get(8);
  if ((cmf & 15u) != 8u || (cmf >> 4) > 7u || ((cmf << 8) | flg) % 31u != 0u || (flg & 0x20u)) st = kErrHeader;
  bool last = st != kOk;
  while (!last) {
    last = br.get(1) != 0u;
    const uint32_t type = br.get(2);
    if (type == 0u) {  // stored
      br.align_byte();
      const uint32_t L = br.get(16), NL = br.get(16);
      if ((L ^ 0xFFFFu) != NL) {
        st = kErrStored;
        break;
      }
      // the bit buffer holds whole bytes now: drain it first, then copy
      uint32_t k = 0;
      for (; k < L && br.n >= 8u; k++) {
        if (o >= d.cap) break;
        out[o++] = (uint8_t)br.get(8);
      }
      if (k < L) {
        if (o + (L - k) > d.cap) {
          st = kErrOutput;
          break;
        }
        if (br.p + (L - k) > br.end) {
          st = kErrInput;
          break;
        }
        copy_bytes(out + o, br.p, L - k);
        o += L - k;
        br.p += L - k;
      }
      if (br.overrun()) {
        st = kErrInput;
        break;
      }
      continue;
    }
    if (type == 3u) {
      st = kErrCode;
      break;
    }
    if (type == 1u) {  // fixed codes (RFC 1951 §3.2.6)
      for (int s = 0; s < 144; s++) T.lens[s] = 8;
      for (int s = 144; s < 256; s++) T.lens[s] = 9;
      for (int s = 256; s < 280; s++) T.lens[s] = 7;
      for (int s = 280; s < 288; s++) T.lens[s] = 8;
      construct(T.lc, T.lsym, T.next, T.lens, 288);
      for (int s = 0; s < 30; s++) T.lens[s] = 5;
      construct(T.dc, T.dsym, T.next, T.lens, 30);
    } else {  // dynamic (RFC 1951 §3.2.7)
      const uint32_t nlen = br.get(5) + 257u, ndist = br.get(5) + 1u, ncode = br.get(4) + 4u;
      if (nlen > 286u || ndist > 30u) {
        st = kErrCode;
        break;
      }
      for (int s = 0; s < 19; s++) T.lens[s] = 0;
      for (uint32_t s = 0; s < ncode; s++) T.lens[kOrder[s]] = (uint8_t)br.get(3);
      if (!construct(T.lc, T.lsym, T.next, T.lens, 19)) {
        st = kErrCode;
        break;
      }
      uint32_t idx = 0;
      bool bad = false;
      while (idx < nlen + ndist) {
        int sym = decode(br, T.lc, T.lsym);
        if (sym < 0) {
          bad = true;
          break;
        }
        if (sym < 16) {
          T.lens[idx++] = (uint8_t)sym;
        } else {
          uint32_t rep, v = 0u;
          if (sym == 16) {
            if (idx == 0u) {
              bad = true;
              break;
            }
            v = T.lens[idx - 1u];
            rep = 3u + br.get(2);
          } else if (sym == 17) {
            rep = 3u + br.get(3);
          } else {
            rep = 11u + br.get(7);
          }
          if (idx + rep > nlen + ndist) {
            bad = true;
            break;
          }
          while (rep--) T.lens[idx++] = (uint8_t)v;
        }
      }
      if (bad || T.lens[256] == 0u) {
        st = kErrCode;
        break;
      }
      // distance lengths first (they sit after the literal/length ones in lens)
      for (uint32_t s = 0; s < 30u; s++) T.dlens[s] = s < ndist ? T.lens[nlen + s] : 0u;
      for (uint32_t s = nlen; s < 288u; s++) T.lens[s] = 0u;
      if (!construct(T.lc, T.lsym, T.next, T.lens, 288)) {
        st = kErrCode;
        break;
      }
      if (!construct(T.dc, T.dsym, T.next, T.dlens, 30)) {
        st = kErrCode;
        break;
      }
    }
    // the block's symbols
    for (;;) {
      const int sym = decode(br, T.lc, T.lsym);
      if (sym < 0) {
        st = kErrCode;
        break;
      }
      if (sym < 256) {
        if (o >= d.cap) {
          st = kErrOutput;
          break;
        }
        out[o++] = (uint8_t)sym;
      } else if (sym == 256) {
        break;
      } else {
        const uint32_t ls = (uint32_t)sym - 257u;
        if (ls >= 29u) {
          st = kErrCode;
          break;
        }
        const uint32_t len = len_base(ls) + br.get(len_extra(ls));
        const int ds = decode(br, T.dc, T.dsym);
        if (ds < 0 || ds >= 30) {
          st = kErrCode;
          break;
        }
        const uint32_t dist = dist_base((uint32_t)ds) + br.get(dist_extra((uint32_t)ds));
        if (dist > o) {
          st = kErrDist;
          break;
        }
        if (o + len > d.cap) {
          st = kErrOutput;
          break;
        }
        copy_match(out + o, dist, len);
        o += len;
      }
    }
    if (st != kOk) break;
    if (br.overrun()) {
      st = kErrInput;
      break;
    }
  }
  if (st == kOk) {  // Adler-32 trailer (RFC 1950 §2.2), checked against the output
    br.align_byte();
    const uint32_t a1 = br.get(8), a2 = br.get(8), a3 = br.get(8), a4 = br.get(8);
    const uint32_t want = (a1 << 24) | (a2 << 16) | (a3 << 8) | a4;
    if (br.overrun()) {
      st = kErrInput;
    } else {
      uint32_t a = 1u, b = 0u;
      for (uint32_t j = 0; j < o;) {
        const uint32_t stop = min(o, j + 5552u);  // zlib's NMAX: no overflow before the modulo
        for (; j < stop; j++) {
          a += out[j];
          b += a;
        }
        a %= 65521u;
        b %= 65521u;
      }
      if (((b << 16) | a) != want) st = kErrHeader;
    }
  }
  out_len[i] = o;
  status[i] = st;
}

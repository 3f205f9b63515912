// hbx_inflate.hip — zlib inflate on gfx950, one wave per stream (the read
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
// A stream is serial in its bits, not in its bytes: lane 0 decodes symbols
// (canonical Huffman, RFC 1951 §3.2.2, through a 9-bit first-level table)
// into a token list, and the whole wave writes them — literal runs one byte
// per lane, matches 64 bytes per step out of a 32 KiB output ring in LDS.
// The input is staged into LDS by the wave.  (Round 1 ran one stream per
// LANE: 64 streams diverging in one wave, byte loads on the bit reader's
// critical path; 0.14 GB/s on 272 long text streams.)  Every read and write
// is bounds-checked: a corrupt stream sets its status and stops, it never
// touches memory outside its input and output.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace hbxi {

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

__device__ const uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                          31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__device__ const uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

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

}  // namespace hbxi

struct InflateDesc {
  uint64_t src;   // device address of the zlib stream
  uint64_t dst;   // device address of the output
  uint32_t len;   // stream bytes
  uint32_t cap;   // output capacity
};

namespace hbxi {

constexpr uint32_t kWin = 32768;   // RFC 1951 window: the output ring in LDS
constexpr uint32_t kInBuf = 4096;  // staged input bytes (+16 slack)
constexpr uint32_t kTok = 512;     // tokens per decode batch
constexpr uint32_t kLutBits = 9;   // first-level decode table
constexpr uint32_t kAdlerMod = 65521u;
// why lane 0 handed the batch back
constexpr uint32_t kNeedInput = 1, kEndOfBlock = 2, kTokFull = 3;

// One wave per stream (64 threads = one workgroup).  Lane 0 reads bits and
// decodes symbols into a token list; the whole wave then writes the output:
// literal runs one byte per lane, matches 64 bytes per step from the 32 KiB
// output ring in LDS (a distance below 64 repeats the pattern by lane mod
// distance), each byte to the ring and to global memory (consecutive bytes
// per wave instruction), and each lane folds its bytes into the Adler-32
// partial sums.  The input is staged into LDS 4 KiB at a time by the wave.
struct WaveInflate {
  uint8_t ring[kWin];
  uint8_t in[kInBuf + 16];
  uint32_t tok[kTok];
  Code lc, dc;
  uint16_t lsym[kLenSyms], dsym[kDistSyms];
  uint16_t llut[1u << kLutBits], dlut[1u << kLutBits];  // (symbol << 4) | length, 0 = longer than 9 bits
  uint8_t lens[320], dlens[32];
  uint16_t next[16];
};

// First-level table entry for the 9 stream bits e (first-sent bit = bit 0).
__device__ __forceinline__ uint16_t lut_entry(const Code& c, const uint16_t* sym, uint32_t e) {
  const uint32_t rev = __builtin_bitreverse32(e) >> (32u - kLutBits);  // first-sent bit on top
  for (uint32_t l = 1; l <= kLutBits; l++) {
    const uint32_t prefix = rev >> (kLutBits - l);
    if (prefix < c.limit[l]) return (uint16_t)((sym[(int)prefix + c.base[l]] << 4) | l);
  }
  return 0;
}

// Lane 0's bit reader over the staged input: byte q of the stream is
// in[q - base] (zero past the stream's end).
struct WaveBits {
  uint64_t buf;
  uint32_t n;
  uint64_t p;  // next stream byte to load
  // Top the buffer up to >= 57 bits with ONE unaligned 8-byte read (two
  // aligned LDS reads).  Bits of a partly fitting byte land above the count
  // too; the next fill ORs the same byte onto them, so they are harmless.
  __device__ __forceinline__ void fill(const uint8_t* in, uint64_t base, uint64_t len) {
    if (n > 56u) return;
    const uint64_t q = p - base;
    uint64_t v = 0ull;
    // the staging keeps p inside the window; outside it (a corrupt stream
    // the headroom checks did not foresee) zeros are read and the stream
    // then fails its overrun or Adler check
    if (q + 16u <= kInBuf + 16u) {
      const uint64_t* w = reinterpret_cast<const uint64_t*>(in + (q & ~7ull));
      const uint32_t sh = (uint32_t)(q & 7u) * 8u;
      v = sh ? (w[0] >> sh) | (w[1] << (64u - sh)) : w[0];
    }
    if (p + 8u > len) {  // zeros past the end of the stream
      const uint64_t keep = len > p ? len - p : 0ull;
      v &= keep ? (~0ull >> (64u - 8u * (uint32_t)keep)) : 0ull;
    }
    const uint32_t take = (64u - n) >> 3;
    buf |= v << n;
    p += take;
    n += 8u * take;
  }
  __device__ __forceinline__ uint32_t get(uint32_t k, const uint8_t* in, uint64_t base, uint64_t len) {
    if (n < k) fill(in, base, len);
    const uint32_t v = (uint32_t)(buf & ((1ull << k) - 1ull));
    buf >>= k;
    n -= k;
    return v;
  }
  // bytes of the stream consumed so far (whole bytes still in buf excluded)
  __device__ __forceinline__ uint64_t byte_pos() const { return p - (n >> 3); }
};

__device__ __forceinline__ int wave_decode(WaveBits& br, const Code& c, const uint16_t* sym, const uint16_t* lut,
                                           const uint8_t* in, uint64_t base, uint64_t len) {
  if (br.n < 15u) br.fill(in, base, len);
  const uint32_t e = lut[br.buf & ((1u << kLutBits) - 1u)];
  if (e) {
    const uint32_t l = e & 15u;
    br.buf >>= l;
    br.n -= l;
    return (int)(e >> 4);
  }
  const uint32_t peek = __builtin_bitreverse32((uint32_t)br.buf) >> 17;
  for (uint32_t l = kLutBits + 1; l <= 15u; l++) {
    const uint32_t prefix = peek >> (15u - l);
    if (prefix < c.limit[l]) {
      br.buf >>= l;
      br.n -= l;
      return sym[(int)prefix + c.base[l]];
    }
  }
  return -1;
}

// The same reader run by the whole wave in lockstep on uniform (scalar)
// values: every LDS value it reads is made uniform with readfirstlane, so
// its state lives in SGPRs and its branches are scalar (no exec-mask
// bookkeeping, which dominated the lane-0 loop: PMC ~50 SALU per token).
__device__ __forceinline__ uint32_t ufirst(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t ufirst64(uint64_t v) {
  return ((uint64_t)ufirst((uint32_t)(v >> 32)) << 32) | ufirst((uint32_t)v);
}

struct UBits {
  uint64_t buf;
  uint32_t n;
  uint32_t p;  // next stream byte to load (streams are < 4 GiB)
  __device__ __forceinline__ void fill(const uint8_t* in, uint32_t base, uint32_t len) {
    if (n > 56u) return;
    const uint32_t q = p - base;
    uint64_t v = 0ull;
    if (q <= kInBuf) {  // (see WaveBits::fill)
      const uint64_t* w = reinterpret_cast<const uint64_t*>(in + (q & ~7u));
      const uint32_t sh = (q & 7u) * 8u;
      const uint64_t w0 = ufirst64(w[0]), w1 = ufirst64(w[1]);
      v = sh ? (w0 >> sh) | (w1 << (64u - sh)) : w0;
    }
    if (p + 8u > len) {
      const uint32_t keep = len > p ? len - p : 0u;
      v &= keep ? (~0ull >> (64u - 8u * keep)) : 0ull;
    }
    const uint32_t take = (64u - n) >> 3;
    buf |= v << n;
    p += take;
    n += 8u * take;
  }
  __device__ __forceinline__ uint32_t get(uint32_t k, const uint8_t* in, uint32_t base, uint32_t len) {
    if (n < k) fill(in, base, len);
    const uint32_t v = (uint32_t)(buf & ((1ull << k) - 1ull));
    buf >>= k;
    n -= k;
    return v;
  }
};

__device__ __forceinline__ int u_decode(UBits& br, const Code& c, const uint16_t* sym, const uint16_t* lut,
                                        const uint8_t* in, uint32_t base, uint32_t len) {
  if (br.n < 15u) br.fill(in, base, len);
  const uint32_t e = ufirst(lut[br.buf & ((1u << kLutBits) - 1u)]);
  if (e) {
    const uint32_t l = e & 15u;
    br.buf >>= l;
    br.n -= l;
    return (int)(e >> 4);
  }
  const uint32_t peek = __builtin_bitreverse32((uint32_t)br.buf) >> 17;
  for (uint32_t l = kLutBits + 1; l <= 15u; l++) {
    const uint32_t prefix = peek >> (15u - l);
    if (prefix < ufirst(c.limit[l])) {
      br.buf >>= l;
      br.n -= l;
      return (int)ufirst(sym[(int)prefix + (int16_t)ufirst((uint32_t)(uint16_t)c.base[l])]);
    }
  }
  return -1;
}

__device__ __forceinline__ uint64_t bcast64(uint64_t v) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}
__device__ __forceinline__ uint32_t bcast32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

}  // namespace hbxi

// One workgroup (one wave) per stream.  out_len[i] = inflated bytes,
// status[i] = 0 or an hbxi::kErr* code.
extern "C" __global__ __launch_bounds__(64) void hbx_k8_inflate(const InflateDesc* __restrict__ desc, uint32_t n,
                                                                 uint32_t* __restrict__ out_len,
                                                                 uint32_t* __restrict__ status) {
  using namespace hbxi;
  __shared__ WaveInflate W;
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  const uint32_t lane = threadIdx.x;
  const InflateDesc d = desc[i];
  const uint8_t* src = reinterpret_cast<const uint8_t*>(d.src);
  uint8_t* out = reinterpret_cast<uint8_t*>(d.dst);
  const uint64_t len = d.len, cap = d.cap;
  uint64_t base = 0;  // stream offset of W.in[0] (uniform)
  // stage input bytes [at, at + kInBuf + 16) (zeros past the end)
  auto stage = [&](uint64_t at) {
    __syncthreads();
    for (uint32_t k = lane * 16u; k < kInBuf + 16u; k += 1024u) {
      if (at + k + 16u <= len) {
        *reinterpret_cast<uint4*>(W.in + k) = *reinterpret_cast<const uint4*>(src + at + k);
      } else {
#pragma unroll
        for (uint32_t q = 0; q < 16u; q++) W.in[k + q] = at + k + q < len ? src[at + k + q] : (uint8_t)0;
      }
    }
    base = at;
    __syncthreads();
  };
  WaveBits br{0ull, 0u, 0ull};  // meaningful in lane 0
  uint64_t o = 0;               // output bytes written (uniform)
  uint32_t st = kOk;            // uniform after each broadcast
  uint32_t s0 = 0u;             // Adler partial sums of this lane's bytes:
  uint64_t s1 = 0ull;           // sum x, sum pos * x
  uint64_t steps = 0;
  auto put = [&](uint64_t pos, uint32_t b) {
    W.ring[pos & (kWin - 1u)] = (uint8_t)b;
    out[pos] = (uint8_t)b;
    s0 += b;
    s1 += pos * (uint64_t)b;
  };
  auto step_done = [&]() {
    if ((++steps & 0xFFFFFull) == 0ull) {  // keep the sums far from overflow
      s0 %= kAdlerMod;
      s1 %= kAdlerMod;
    }
  };
  // write tokens [0, nt) (all lanes).  Tokens come off LDS 64 at a time,
  // one per lane; the wave walks them from registers (readlane / shuffle),
  // so a token costs no dependent LDS round trip of its own.
  auto expand_chunk = [&](uint32_t mytok, uint32_t cn) {  // cn tokens, token t in lane t
    const uint64_t litmask = __builtin_amdgcn_ballot_w64(lane < cn && (mytok >> 31) != 0u);
    uint32_t t = 0;
    while (t < cn) {
      if ((litmask >> t) & 1ull) {  // a run of literals, one per lane
        const uint64_t rest = ~(litmask >> t);
        const uint32_t run = min(rest ? (uint32_t)__builtin_ctzll(rest) : 64u - t, cn - t);
        const uint32_t b = (uint32_t)__shfl((int)mytok, (int)(t + lane), 64) & 0xFFu;
        if (lane < run) put(o + lane, b);
        o += run;
        t += run;
        step_done();
        continue;
      }
      const uint32_t tk = (uint32_t)__builtin_amdgcn_readlane((int)mytok, (int)t);
      const uint32_t L = tk >> 16, D = tk & 0xFFFFu ? tk & 0xFFFFu : 65536u;
      if (D >= 64u) {
        for (uint32_t j0 = 0; j0 < L; j0 += 64u) {
          const uint32_t j = j0 + lane;
          if (j < L) put(o + j, W.ring[(o - D + j) & (kWin - 1u)]);
          step_done();
        }
      } else {  // pattern of period D: byte j = byte (j mod D) of the last D
        const float rD = __builtin_amdgcn_rcpf((float)D);
        auto mod_small = [&](uint32_t x) {  // x mod D for x < 2^12: a reciprocal, one correction
          uint32_t r = x - D * (uint32_t)((float)x * rD);
          return r >= D ? r - D : r;
        };
        const uint32_t m = mod_small(lane), r64 = mod_small(64u);
        uint32_t c = 0;
        for (uint32_t j0 = 0; j0 < L; j0 += 64u) {
          const uint32_t j = j0 + lane;
          uint32_t k = c + m;
          if (k >= D) k -= D;
          if (j < L) put(o + j, W.ring[(o - D + k) & (kWin - 1u)]);
          c += r64;
          if (c >= D) c -= D;
          step_done();
        }
      }
      o += L;
      t++;
    }
  };
  auto expand = [&](uint32_t nt) {  // tokens [0, nt) from W.tok
    for (uint32_t t0 = 0; t0 < nt; t0 += 64u) {
      const uint32_t cn = min(64u, nt - t0);
      expand_chunk(lane < cn ? W.tok[t0 + lane] : 0u, cn);
    }
  };

  stage(0);
  if (lane == 0) {  // zlib header (RFC 1950 §2.2): deflate, window <= 32 KiB, check bits, no dictionary
    const uint32_t cmf = br.get(8, W.in, base, len), flg = br.get(8, W.in, base, len);
    if ((cmf & 15u) != 8u || (cmf >> 4) > 7u || ((cmf << 8) | flg) % 31u != 0u || (flg & 0x20u)) st = kErrHeader;
  }
  st = bcast32(st);
  bool last = st != kOk;
  while (!last) {
    // room for a block header (a dynamic one is < 320 bytes)
    {
      const uint64_t bp = bcast64(br.p);
      if (bp + 512u > base + kInBuf && base + kInBuf < len + 16u) stage(bp & ~15ull);
    }
    uint32_t type = 0, rem = 0, ntok = 0;
    if (lane == 0) {
      last = br.get(1, W.in, base, len) != 0u;
      type = br.get(2, W.in, base, len);
      if (type == 0u) {  // stored: the whole bytes left in the bit buffer, then the rest straight from the input
        br.buf >>= (br.n & 7u);
        br.n -= br.n & 7u;
        const uint32_t SL = br.get(16, W.in, base, len), NL = br.get(16, W.in, base, len);
        if ((SL ^ 0xFFFFu) != NL) {
          st = kErrStored;
        } else {
          uint32_t k = 0;
          for (; k < SL && br.n >= 8u && st == kOk; k++) {
            if (o + k >= cap) st = kErrOutput;
            else W.tok[ntok++] = 0x80000000u | br.get(8, W.in, base, len);
          }
          rem = SL - k;
          if (st == kOk && rem) {
            if (o + k + rem > cap) st = kErrOutput;
            else if (br.p + rem > len) st = kErrInput;
          }
        }
      } else if (type == 3u) {
        st = kErrCode;
      } else if (type == 1u) {  // fixed codes (RFC 1951 §3.2.6)
        for (int s = 0; s < 144; s++) W.lens[s] = 8;
        for (int s = 144; s < 256; s++) W.lens[s] = 9;
        for (int s = 256; s < 280; s++) W.lens[s] = 7;
        for (int s = 280; s < 288; s++) W.lens[s] = 8;
        construct(W.lc, W.lsym, W.next, W.lens, 288);
        for (int s = 0; s < 30; s++) W.dlens[s] = 5;
        construct(W.dc, W.dsym, W.next, W.dlens, 30);
      } else {  // dynamic (RFC 1951 §3.2.7)
        const uint32_t nlen = br.get(5, W.in, base, len) + 257u, ndist = br.get(5, W.in, base, len) + 1u,
                       ncode = br.get(4, W.in, base, len) + 4u;
        if (nlen > 286u || ndist > 30u) st = kErrCode;
        if (st == kOk) {
          for (int s = 0; s < 19; s++) W.lens[s] = 0;
          for (uint32_t s = 0; s < ncode; s++) W.lens[kOrder[s]] = (uint8_t)br.get(3, W.in, base, len);
          if (!construct(W.lc, W.lsym, W.next, W.lens, 19)) st = kErrCode;
        }
        uint32_t idx = 0;
        while (st == kOk && idx < nlen + ndist) {
          if (br.n < 15u) br.fill(W.in, base, len);
          const uint32_t peek = __builtin_bitreverse32((uint32_t)br.buf) >> 17;
          int sym = -1;
          for (uint32_t l = 1; l <= 15u; l++) {
            const uint32_t prefix = peek >> (15u - l);
            if (prefix < W.lc.limit[l]) {
              br.buf >>= l;
              br.n -= l;
              sym = W.lsym[(int)prefix + W.lc.base[l]];
              break;
            }
          }
          if (sym < 0) {
            st = kErrCode;
          } else if (sym < 16) {
            W.lens[idx++] = (uint8_t)sym;
          } else {
            uint32_t rep, v = 0u;
            if (sym == 16) {
              if (idx == 0u) st = kErrCode;
              v = idx ? W.lens[idx - 1u] : 0u;
              rep = 3u + br.get(2, W.in, base, len);
            } else if (sym == 17) {
              rep = 3u + br.get(3, W.in, base, len);
            } else {
              rep = 11u + br.get(7, W.in, base, len);
            }
            if (idx + rep > nlen + ndist) st = kErrCode;
            while (st == kOk && rep--) W.lens[idx++] = (uint8_t)v;
          }
        }
        if (st == kOk && W.lens[256] == 0u) st = kErrCode;
        if (st == kOk) {
          for (uint32_t s = 0; s < 30u; s++) W.dlens[s] = s < ndist ? W.lens[nlen + s] : 0u;
          for (uint32_t s = nlen; s < 288u; s++) W.lens[s] = 0u;
          if (!construct(W.lc, W.lsym, W.next, W.lens, 288) || !construct(W.dc, W.dsym, W.next, W.dlens, 30))
            st = kErrCode;
        }
      }
    }
    __syncthreads();
    st = bcast32(st);
    last = bcast32(last ? 1u : 0u) != 0u;
    type = bcast32(type);
    if (st != kOk) break;
    if (type == 0u) {  // stored
      ntok = bcast32(ntok);
      rem = bcast32(rem);
      expand(ntok);
      const uint64_t at = bcast64(br.p);
      for (uint32_t j0 = 0; j0 < rem; j0 += 64u) {
        const uint32_t j = j0 + lane;
        if (j < rem) put(o + j, src[at + j]);
        step_done();
      }
      o += rem;
      if (lane == 0) br.p += rem;
      continue;  // the next block header restages the input
    }
    // Huffman block: first-level tables by the whole wave, then the symbols
    for (uint32_t e = lane; e < (1u << kLutBits); e += 64u) {
      W.llut[e] = lut_entry(W.lc, W.lsym, e);
      W.dlut[e] = lut_entry(W.dc, W.dsym, e);
    }
    __syncthreads();
    // the symbols: the whole wave decodes in lockstep on uniform values, 64
    // tokens at a time into a register (token t in lane t), then writes them
    UBits ub{bcast64(br.buf), bcast32(br.n), (uint32_t)bcast64(br.p)};
    const uint32_t len32 = (uint32_t)len;
    for (;;) {
      const uint32_t b32 = (uint32_t)base;
      // past lim the next token could need bytes beyond the staged window
      const uint32_t lim = base + kInBuf < len + 16u ? b32 + kInBuf - 16u : 0xFFFFFFFFu;
      uint32_t toks = 0, cnt = 0, why = 0;
      uint64_t ov = o;  // output including this chunk's tokens
      while (cnt < 64u) {
        if (ub.p > lim) {
          why = kNeedInput;
          break;
        }
        const int sym = u_decode(ub, W.lc, W.lsym, W.llut, W.in, b32, len32);
        uint32_t tv;
        if (sym < 0) {
          st = kErrCode;
          break;
        }
        if (sym < 256) {
          if (ov >= cap) {
            st = kErrOutput;
            break;
          }
          tv = 0x80000000u | (uint32_t)sym;
          ov++;
        } else if (sym == 256) {
          why = kEndOfBlock;
          break;
        } else {
          const uint32_t ls = (uint32_t)sym - 257u;
          if (ls >= 29u) {
            st = kErrCode;
            break;
          }
          const uint32_t L = len_base(ls) + ub.get(len_extra(ls), W.in, b32, len32);
          const int ds = u_decode(ub, W.dc, W.dsym, W.dlut, W.in, b32, len32);
          if (ds < 0 || ds >= 30) {
            st = kErrCode;
            break;
          }
          const uint32_t D = dist_base((uint32_t)ds) + ub.get(dist_extra((uint32_t)ds), W.in, b32, len32);
          if (D > ov) {
            st = kErrDist;
            break;
          }
          if (ov + L > cap) {
            st = kErrOutput;
            break;
          }
          tv = (L << 16) | (D & 0xFFFFu);  // D = 32768 is stored as 0x8000; never 0
          ov += L;
        }
        toks = lane == cnt ? tv : toks;
        cnt++;
      }
      if (st != kOk) break;
      expand_chunk(toks, cnt);
      if (why == kEndOfBlock) break;
      if (why == kNeedInput) stage(ub.p & ~15u);
    }
    br.buf = ub.buf;  // lane 0's reader takes over for the next block header
    br.n = ub.n;
    br.p = ub.p;
    if (st != kOk) break;
    if (lane == 0) {  // consumed past the input?
      if (8ull * br.p - br.n > 8ull * len) st = kErrInput;
    }
    st = bcast32(st);
    if (st != kOk) break;
  }
  if (st == kOk) {  // Adler-32 trailer (RFC 1950 §2.2) against the sums of the bytes written
    const uint64_t bp = bcast64(br.p);
    if (bp + 16u > base + kInBuf) stage(bp & ~15ull);
    uint32_t want = 0;
    if (lane == 0) {
      br.buf >>= (br.n & 7u);
      br.n -= br.n & 7u;
      const uint32_t a1 = br.get(8, W.in, base, len), a2 = br.get(8, W.in, base, len),
                     a3 = br.get(8, W.in, base, len), a4 = br.get(8, W.in, base, len);
      want = (a1 << 24) | (a2 << 16) | (a3 << 8) | a4;
      if (8ull * br.p - br.n > 8ull * len) st = kErrInput;
    }
    st = bcast32(st);
    want = bcast32(want);
    uint32_t a = s0 % kAdlerMod, b = (uint32_t)(s1 % kAdlerMod);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      a += (uint32_t)__shfl_xor((int)a, off, 64);
      b += (uint32_t)__shfl_xor((int)b, off, 64);
      a %= kAdlerMod;
      b %= kAdlerMod;
    }
    const uint64_t om = o % kAdlerMod;
    const uint32_t A = (uint32_t)((1u + a) % kAdlerMod);
    const uint32_t B = (uint32_t)((om + om * a + kAdlerMod - b) % kAdlerMod);
    if (st == kOk && ((B << 16) | A) != want) st = kErrHeader;
  }
  if (lane == 0) {
    out_len[i] = (uint32_t)o;
    status[i] = st;
  }
}

// ---- lane per stream (many short compressible streams) ----
// 64 streams per wave: the decode diverges but 64 streams progress per
// instruction stream, which wins when there are tens of thousands of short
// compressible streams (65,536 x 16 KiB text: 13 GB/s vs 4.8 for a wave per
// stream); the wave per stream wins everywhere else (stored and long
// streams).  hbx_inflate_blocks_device picks one per call.
namespace hbxi {
struct LaneTables {
  Code lc, dc;
  uint16_t next[16];  // placement cursors while a table is built
  uint16_t lsym[kLenSyms];
  uint16_t dsym[kDistSyms];
  uint8_t lens[320];  // code lengths while a dynamic table is built
  uint8_t dlens[32];
};

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

// One lane per stream.  out_len[i] = inflated bytes, status[i] = 0 or an
// hbxi::kErr* code.
extern "C" __global__ __launch_bounds__(64) void hbx_k8_inflate_lanes(const InflateDesc* __restrict__ desc, uint32_t n,
                                                                 uint32_t* __restrict__ out_len,
                                                                 uint32_t* __restrict__ status) {
  using namespace hbxi;
  __shared__ LaneTables tabs[64];
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

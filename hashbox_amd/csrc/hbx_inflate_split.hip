// hbx_inflate_split.hip — inflate of a few LONG compressible zlib streams,
// parallel within each stream (K8s).
//
// Reference: the same UncompressData before VerifyBlock as hbx_inflate.hip
// (pkg/core/block.go:113-131, 186-201; restore hashback/restore.go:51-52).
// One wave decodes one stream at ~4 MB/s (a chain of dependent table reads
// per symbol), so 272 streams of 4 MiB leave most of the 1,024 SIMDs idle and
// the device is slower than 16 host threads.  Here each stream's compressed
// bytes are cut into regions of kSplitRegion bytes and decoded by one wave per
// region at once, rapidgzip-style:
//
//   K8s-find     (one wave per region k >= 1): the first bit position in the
//                region where a deflate block can start: a dynamic-Huffman
//                header that parses completely and is valid the way zlib
//                checks it (complete code-length code, code lengths that fit,
//                end-of-block code present, complete literal/length and
//                distance codes), or the byte right after a sync flush
//                (00 00 FF FF, the empty stored block that ends every piece of
//                a K7 stream).  Region 0 starts after the zlib header.
//   K8s-decode   (one wave per region): from the region's start, whole
//                blocks until the first block end at or past the NEXT
//                region's start (or the final block), into 16-bit symbols: a
//                literal byte, or a MARKER 0x8000 | w for "byte w of the
//                32 KiB window before this region's output" (a back-reference
//                reaching before the region's first symbol; copies of markers
//                stay markers).  The wave keeps the last kRing symbols in LDS;
//                older in-region sources are read back from the scratch
//                (flushed first).
//   K8s-resolve  (one workgroup per stream): walks the chain region 0 ->
//                the region whose start equals the previous one's end ->
//                ..., writes the bytes (markers from the output already
//                written), folds Adler-32 and checks the trailer.
//
// Nothing here decides a result on its own: a stream whose chain does not
// close exactly (a false start, a region whose symbols overflow its scratch,
// any decode error, a bad trailer) is flagged, and the engine inflates it
// again with the sequential kernel (hbx_k8_inflate), which also produces the
// exact error status of a corrupt stream.  So the split path only ever
// reports streams it decoded completely and verified by Adler-32.
#pragma once

#include "hbx_inflate.hip"

// Host-built: one per region of a split stream.
struct SplitRegion {
  uint32_t stream;  // index into the call's InflateDesc array
  uint32_t k;       // region index within the stream
  uint32_t first;   // index of the stream's region 0 in the region array
  uint32_t count;   // regions of the stream
  uint64_t sym;     // this region's scratch offset, in 16-bit symbols
  uint32_t sym_cap; // its scratch capacity (symbols)
  uint32_t pad;
};
// Written by K8s-decode.
struct SplitResult {
  uint64_t end_bit;  // bit position after the last block decoded
  uint32_t nsym;     // symbols written
  uint32_t flags;    // bit 0: the last block was final; bits 8..15: status (0 = ok)
};

namespace hbxs {

using namespace hbxi;

constexpr uint32_t kSplitRegion = 32768;           // compressed bytes per region
constexpr uint64_t kNoStart = ~0ull;
constexpr uint32_t kRing = 16384;                  // symbols of history in LDS
constexpr uint32_t kStNoStart = 1, kStOverflow = 2, kStBad = 3;  // SplitResult status

// Bytes [p, p + 8) of a stream of `len` bytes, zero past its end.
__device__ __forceinline__ uint64_t ld64(const uint8_t* src, uint64_t len, uint64_t p) {
  if (p + 8u <= len)  // an 8-byte load at any byte address (unaligned access: the hardware splits it)
    return *reinterpret_cast<const __attribute__((address_space(1))) uint64_t*>(
        reinterpret_cast<uintptr_t>(src + p));
  uint64_t v = 0ull;
  for (uint32_t q = 0; q < 8u && p + q < len; q++) v |= (uint64_t)src[p + q] << (8u * q);
  return v;
}

// A per-lane bit reader straight from global memory (the find kernel's full
// header check, rare and divergent).
struct GBits {
  const uint8_t* src;
  uint64_t len;
  uint64_t p;  // next byte to load
  uint64_t buf;
  uint32_t n;
  __device__ __forceinline__ void skip_to(uint64_t bit) {
    p = bit >> 3;
    buf = 0ull;
    n = 0u;
    fill();
    const uint32_t k = (uint32_t)(bit & 7u);
    buf >>= k;
    n -= k;
  }
  __device__ __forceinline__ void fill() {
    if (n > 56u) return;
    const uint64_t v = ld64(src, len, p);
    const uint32_t take = (64u - n) >> 3;
    buf |= v << n;
    p += take;
    n += 8u * take;
  }
  __device__ __forceinline__ uint32_t get(uint32_t k) {
    if (n < k) fill();
    const uint32_t v = (uint32_t)(buf & ((1ull << k) - 1ull));
    buf >>= k;
    n -= k;
    return v;
  }
  __device__ __forceinline__ bool past_end() const { return 8ull * p - n > 8ull * len; }
};

// Does a dynamic block header that zlib would accept start at `bit`?  (RFC
// 1951 §3.2.7; the acceptance rules of zlib's inflate_table: the code-length
// code must be complete, the literal/length and distance codes complete
// unless they hold a single code, symbol 256 must have a code.)
__device__ bool valid_dynamic(const uint8_t* src, uint64_t len, uint64_t bit) {
  GBits br{src, len, 0ull, 0ull, 0u};
  br.skip_to(bit);
  (void)br.get(1);
  if (br.get(2) != 2u) return false;
  const uint32_t nlen = br.get(5) + 257u, ndist = br.get(5) + 1u, ncode = br.get(4) + 4u;
  if (nlen > 286u || ndist > 30u) return false;
  uint64_t cl = 0ull;  // code-length code lengths by symbol, 3 bits each
  uint32_t kraft = 0u;
  for (uint32_t s = 0; s < ncode; s++) {
    const uint32_t l = br.get(3);
    cl |= (uint64_t)l << (3u * kOrder[s]);
    if (l) kraft += 1u << (7u - l);
  }
  if (kraft != 128u) return false;
  // canonical decode of the code-length code: first code and first symbol
  // index per length (lengths 1..7)
  uint32_t count[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t s = 0; s < 19u; s++) count[(cl >> (3u * s)) & 7u]++;
  count[0] = 0;
  uint32_t kl = 0u, kd = 0u, nl = 0u, nd = 0u, prev = 0u;
  bool eob = false;
  for (uint32_t idx = 0; idx < nlen + ndist;) {
    // read one code bit by bit (MSB-first code, LSB-first stream)
    uint32_t code = 0u, first = 0u, index = 0u;
    int sym = -1;
    for (uint32_t l = 1; l <= 7u; l++) {
      code |= br.get(1);
      const uint32_t c = count[l];
      if (code < first + c) {
        // the (code - first)-th symbol of length l in symbol order
        uint32_t r = code - first;
        for (uint32_t s = 0; s < 19u; s++)
          if (((cl >> (3u * s)) & 7u) == l && r-- == 0u) {
            sym = (int)s;
            break;
          }
        break;
      }
      index += c;
      first = (first + c) << 1;
      code <<= 1;
    }
    (void)index;
    if (sym < 0 || br.past_end()) return false;
    uint32_t v, rep;
    if (sym < 16) {
      v = (uint32_t)sym;
      rep = 1u;
    } else if (sym == 16) {
      if (idx == 0u) return false;
      v = prev;
      rep = 3u + br.get(2);
    } else {
      v = 0u;
      rep = sym == 17 ? 3u + br.get(3) : 11u + br.get(7);
    }
    if (idx + rep > nlen + ndist) return false;
    for (uint32_t q = 0; q < rep; q++, idx++) {
      if (idx < nlen) {
        if (v) {
          kl += 1u << (15u - v);
          nl++;
        }
        if (idx == 256u) eob = v != 0u;
      } else if (v) {
        kd += 1u << (15u - v);
        nd++;
      }
    }
    prev = v;
  }
  // zlib accepts an incomplete code only when it is one code of length 1,
  // and a block without distance codes
  if (!eob || kl > 32768u || kd > 32768u) return false;
  if (kl != 32768u && !(nl == 1u && kl == 16384u)) return false;
  if (kd != 32768u && nd != 0u && !(nd == 1u && kd == 16384u)) return false;
  return !br.past_end();
}

}  // namespace hbxs

// K8s-find: the first block start in region k >= 1 of its stream (bit
// position, or kNoStart); region 0 starts after the zlib header (bit 16).
extern "C" __global__ __launch_bounds__(64) void hbx_k8s_find(const InflateDesc* __restrict__ desc,
                                                              const SplitRegion* __restrict__ reg, uint32_t nreg,
                                                              uint64_t* __restrict__ start) {
  using namespace hbxs;
  const uint32_t r = blockIdx.x;
  if (r >= nreg) return;
  const SplitRegion R = reg[r];
  const uint32_t lane = threadIdx.x;
  if (R.k == 0u) {
    if (lane == 0) start[r] = 16u;
    return;
  }
  const InflateDesc d = desc[R.stream];
  const uint8_t* src = reinterpret_cast<const uint8_t*>(d.src);
  const uint64_t len = d.len;
  const uint64_t lo = (uint64_t)R.k * kSplitRegion, hi = min(lo + kSplitRegion, len);
  uint64_t found = kNoStart;
  for (uint64_t p0 = lo; p0 < hi && found == kNoStart; p0 += 64u) {
    const uint64_t p = p0 + lane;
    uint32_t best = 8u;  // the lane's first valid bit offset in byte p
    if (p < hi) {
      const uint64_t w0 = ld64(src, len, p), w1 = ld64(src, len, p + 8u), w2 = ld64(src, len, p + 16u);
      // after a sync flush (00 00 FF FF) the next block starts at this byte
      const uint32_t before = (uint32_t)(ld64(src, len, p - 4u) & 0xFFFFFFFFu);
      if (before == 0xFFFF0000u && ((w0 >> 1) & 3u) != 3u) best = 0u;
      for (uint32_t j = 0; j < 8u && best == 8u; j++) {
        const uint64_t v = j ? (w0 >> j) | (w1 << (64u - j)) : w0;
        const uint64_t v2 = j ? (w1 >> j) | (w2 << (64u - j)) : w1;
        if (((v >> 1) & 3u) != 2u || ((v >> 3) & 31u) > 29u || ((v >> 8) & 31u) > 29u) continue;
        const uint32_t ncode = (uint32_t)((v >> 13) & 15u) + 4u;
        uint32_t kraft = 0u;
        for (uint32_t s = 0; s < ncode; s++) {
          const uint32_t b = 17u + 3u * s;
          const uint32_t l = (uint32_t)((b + 3u <= 64u ? v >> b : b >= 64u ? v2 >> (b - 64u)
                                                                               : (v >> b) | (v2 << (64u - b))) & 7u);
          if (l) kraft += 1u << (7u - l);
        }
        if (kraft != 128u) continue;
        if (valid_dynamic(src, len, 8u * p + j)) best = j;
      }
    }
    const uint64_t hit = __builtin_amdgcn_ballot_w64(best < 8u);
    if (hit) {
      const int L = __builtin_ctzll(hit);
      const uint32_t bj = (uint32_t)__builtin_amdgcn_readlane((int)best, L);
      found = 8u * (p0 + (uint64_t)L) + bj;
    }
  }
  if (lane == 0) start[r] = found;
}

namespace hbxs {

struct alignas(16) SplitLds {
  uint16_t ring[kRing];
  uint8_t in[kInBuf + 16];
  Code lc, dc;
  uint16_t lsym[kLenSyms], dsym[kDistSyms];
  uint16_t llut[1u << kLutBits], dlut[1u << kLutBits];
  uint8_t lens[320], dlens[32];
  uint16_t next[16];
};

}  // namespace hbxs

// K8s-decode: one wave per region.  res[r] = where its decode ended, the
// symbols it wrote, whether it reached the final block, and a status.
extern "C" __global__ __launch_bounds__(64) void hbx_k8s_decode(const InflateDesc* __restrict__ desc,
                                                                const SplitRegion* __restrict__ reg, uint32_t nreg,
                                                                const uint64_t* __restrict__ start,
                                                                uint16_t* __restrict__ scratch,
                                                                SplitResult* __restrict__ res) {
  using namespace hbxs;
  __shared__ SplitLds W;
  const uint32_t r = blockIdx.x;
  if (r >= nreg) return;
  const uint32_t lane = threadIdx.x;
  const SplitRegion R = reg[r];
  const uint64_t s0 = start[r];
  if (s0 == kNoStart) {
    if (lane == 0) res[r] = SplitResult{0ull, 0u, kStNoStart << 8};
    return;
  }
  // decode until the first block end at or past the next region's start
  uint64_t target = ~0ull;
  for (uint32_t q = R.k + 1u; q < R.count; q++) {
    const uint64_t t = start[R.first + q];
    if (t != kNoStart) {
      target = t;
      break;
    }
  }
  const InflateDesc d = desc[R.stream];
  const uint8_t* src = reinterpret_cast<const uint8_t*>(d.src);
  const uint64_t len = d.len;
  uint16_t* out = scratch + R.sym;
  const uint32_t cap = R.sym_cap;
  uint64_t base = 0;
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
  uint32_t o = 0;        // symbols written (uniform)
  uint32_t flushed = 0;  // scratch symbols [0, flushed) are known stored (uniform)
  uint32_t st = 0;
  // Symbol at region position q, read while positions [0, wpos) are written:
  // q < 0 is a marker into the window before the region (q >= -32768); the
  // last kRing positions are in the LDS ring; older ones come back from the
  // scratch, once every store up to them is complete (a wave-wide wait, rare:
  // only distances past the ring need it).
  auto sym_at = [&](int64_t q, uint32_t wpos) -> uint32_t {
    const bool far = q >= 0 && (int64_t)wpos - q > (int64_t)kRing;
    if (__builtin_amdgcn_ballot_w64(far && q >= (int64_t)flushed)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      flushed = wpos;
    }
    if (q < 0) return 0x8000u | (uint32_t)(32768 + q);
    if (!far) return W.ring[q & (kRing - 1u)];
    return out[q];
  };
  auto put = [&](uint32_t pos, uint32_t v) {
    W.ring[pos & (kRing - 1u)] = (uint16_t)v;
    out[pos] = (uint16_t)v;
  };
  // tokens: literal 0x80000000 | byte, match (L << 16) | (D & 0xFFFF)
  auto expand_chunk = [&](uint32_t mytok, uint32_t cn) {
    const uint64_t litmask = __builtin_amdgcn_ballot_w64(lane < cn && (mytok >> 31) != 0u);
    uint32_t t = 0;
    while (t < cn) {
      if ((litmask >> t) & 1ull) {
        const uint64_t rest = ~(litmask >> t);
        const uint32_t run = min(rest ? (uint32_t)__builtin_ctzll(rest) : 64u - t, cn - t);
        const uint32_t b = (uint32_t)__shfl((int)mytok, (int)(t + lane), 64) & 0xFFu;
        if (lane < run) put(o + lane, b);
        o += run;
        t += run;
        continue;
      }
      const uint32_t tk = (uint32_t)__builtin_amdgcn_readlane((int)mytok, (int)t);
      const uint32_t L = tk >> 16, D = tk & 0xFFFFu ? tk & 0xFFFFu : 65536u;
      const int64_t from = (int64_t)o - (int64_t)D;
      if (D >= 64u) {
        for (uint32_t j0 = 0; j0 < L; j0 += 64u) {
          const uint32_t j = j0 + lane;
          const uint32_t v = sym_at(from + j, o + j0);
          if (j < L) put(o + j, v);
        }
      } else {  // period D < 64: symbol j = symbol (j mod D) of the last D
        const uint32_t m = lane % D;
        const uint32_t v = sym_at(from + m, o);  // the pattern, lane l holding symbol l mod D
        for (uint32_t j0 = 0; j0 < L; j0 += 64u) {
          const uint32_t j = j0 + lane;
          const uint32_t k = (j0 % D + m) % D;
          const uint32_t vk = (uint32_t)__shfl((int)v, (int)k, 64);
          if (j < L) put(o + j, vk);
        }
      }
      o += L;
      t++;
    }
  };

  WaveBits br{0ull, 0u, 0ull};
  stage(s0 >> 3 & ~15ull);
  if (lane == 0) {
    br.p = s0 >> 3;
    br.fill(W.in, base, len);
    const uint32_t k = (uint32_t)(s0 & 7u);
    br.buf >>= k;
    br.n -= k;
    if (R.k == 0u) {  // region 0 starts right after a valid zlib header
      const uint32_t cmf = src[0], flg = len > 1 ? src[1] : 0u;
      if (len < 2 || (cmf & 15u) != 8u || (cmf >> 4) > 7u || ((cmf << 8) | flg) % 31u != 0u || (flg & 0x20u))
        st = kStBad;
    }
  }
  st = bcast32(st);
  bool last = false;
  uint64_t e = s0;
  while (st == 0u) {
    {
      const uint64_t bp = bcast64(br.p);
      if (bp + 512u > base + kInBuf && base + kInBuf < len + 16u) stage(bp & ~15ull);
    }
    uint32_t type = 0, rem = 0, ntok = 0;
    if (lane == 0) {
      last = br.get(1, W.in, base, len) != 0u;
      type = br.get(2, W.in, base, len);
      if (type == 0u) {
        br.buf >>= (br.n & 7u);
        br.n -= br.n & 7u;
        const uint32_t SL = br.get(16, W.in, base, len), NL = br.get(16, W.in, base, len);
        if ((SL ^ 0xFFFFu) != NL) st = kStBad;
        else {
          // the stored bytes: whole bytes still in the bit buffer, then the rest
          // straight from the input (p is byte-exact once the buffer is empty)
          ntok = min(SL, br.n >> 3);
          rem = SL - ntok;
          if (o + SL > cap) st = kStOverflow;
          else if (br.byte_pos() + SL > len) st = kStBad;
        }
      } else if (type == 3u) {
        st = kStBad;
      } else if (type == 1u) {
        for (int s = 0; s < 144; s++) W.lens[s] = 8;
        for (int s = 144; s < 256; s++) W.lens[s] = 9;
        for (int s = 256; s < 280; s++) W.lens[s] = 7;
        for (int s = 280; s < 288; s++) W.lens[s] = 8;
        construct(W.lc, W.lsym, W.next, W.lens, 288);
        for (int s = 0; s < 30; s++) W.dlens[s] = 5;
        construct(W.dc, W.dsym, W.next, W.dlens, 30);
      } else {
        const uint32_t nlen = br.get(5, W.in, base, len) + 257u, ndist = br.get(5, W.in, base, len) + 1u,
                       ncode = br.get(4, W.in, base, len) + 4u;
        if (nlen > 286u || ndist > 30u) st = kStBad;
        if (st == 0u) {
          for (int s = 0; s < 19; s++) W.lens[s] = 0;
          for (uint32_t s = 0; s < ncode; s++) W.lens[kOrder[s]] = (uint8_t)br.get(3, W.in, base, len);
          if (!construct(W.lc, W.lsym, W.next, W.lens, 19)) st = kStBad;
        }
        uint32_t idx = 0;
        while (st == 0u && idx < nlen + ndist) {
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
            st = kStBad;
          } else if (sym < 16) {
            W.lens[idx++] = (uint8_t)sym;
          } else {
            uint32_t rep, v = 0u;
            if (sym == 16) {
              if (idx == 0u) st = kStBad;
              v = idx ? W.lens[idx - 1u] : 0u;
              rep = 3u + br.get(2, W.in, base, len);
            } else if (sym == 17) {
              rep = 3u + br.get(3, W.in, base, len);
            } else {
              rep = 11u + br.get(7, W.in, base, len);
            }
            if (idx + rep > nlen + ndist) st = kStBad;
            while (st == 0u && rep--) W.lens[idx++] = (uint8_t)v;
          }
        }
        if (st == 0u && W.lens[256] == 0u) st = kStBad;
        if (st == 0u) {
          for (uint32_t s = 0; s < 30u; s++) W.dlens[s] = s < ndist ? W.lens[nlen + s] : 0u;
          for (uint32_t s = nlen; s < 288u; s++) W.lens[s] = 0u;
          if (!construct(W.lc, W.lsym, W.next, W.lens, 288) || !construct(W.dc, W.dsym, W.next, W.dlens, 30))
            st = kStBad;
        }
      }
    }
    __syncthreads();
    st = bcast32(st);
    last = bcast32(last ? 1u : 0u) != 0u;
    type = bcast32(type);
    if (st != 0u) break;
    if (type == 0u) {  // stored: the buffered bytes, then the rest from the input
      ntok = bcast32(ntok);
      rem = bcast32(rem);
      if (lane == 0)  // the <= 8 bytes still in the bit buffer (W.lens as scratch:
        for (uint32_t q = 0; q < ntok; q++) W.lens[q] = (uint8_t)br.get(8, W.in, base, len);  // no table is live)
      __syncthreads();
      if (lane < ntok) put(o + lane, W.lens[lane]);
      o += ntok;
      __syncthreads();
      const uint64_t at = bcast64(br.p);
      for (uint32_t j0 = 0; j0 < rem; j0 += 64u) {
        const uint32_t j = j0 + lane;
        if (j < rem) put(o + j, src[at + j]);
      }
      o += rem;
      if (lane == 0) br.p += rem;
    } else {
      for (uint32_t en = lane; en < (1u << kLutBits); en += 64u) {
        W.llut[en] = lut_entry(W.lc, W.lsym, en);
        W.dlut[en] = lut_entry(W.dc, W.dsym, en);
      }
      __syncthreads();
      UBits ub{bcast64(br.buf), bcast32(br.n), (uint32_t)bcast64(br.p)};
      const uint32_t len32 = (uint32_t)len;
      for (;;) {
        const uint32_t b32 = (uint32_t)base;
        const uint32_t lim = base + kInBuf < len + 16u ? b32 + kInBuf - 16u : 0xFFFFFFFFu;
        uint32_t toks = 0, cnt = 0, why = 0;
        uint64_t ov = o;
        while (cnt < 64u) {
          if (ub.p > lim) {
            why = kNeedInput;
            break;
          }
          const int sym = u_decode(ub, W.lc, W.lsym, W.llut, W.in, b32, len32);
          uint32_t tv;
          if (sym < 0) {
            st = kStBad;
            break;
          }
          if (sym < 256) {
            if (ov >= cap) {
              st = kStOverflow;
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
              st = kStBad;
              break;
            }
            const uint32_t L = len_base(ls) + ub.get(len_extra(ls), W.in, b32, len32);
            const int ds = u_decode(ub, W.dc, W.dsym, W.dlut, W.in, b32, len32);
            if (ds < 0 || ds >= 30) {
              st = kStBad;
              break;
            }
            const uint32_t D = dist_base((uint32_t)ds) + ub.get(dist_extra((uint32_t)ds), W.in, b32, len32);
            // a reference before the region's first symbol is a marker into
            // the 32 KiB window before it; region 0 has no window
            if (D > ov + (R.k ? 32768u : 0u)) {
              st = kStBad;
              break;
            }
            if (ov + L > cap) {
              st = kStOverflow;
              break;
            }
            tv = (L << 16) | (D & 0xFFFFu);
            ov += L;
          }
          toks = lane == cnt ? tv : toks;
          cnt++;
        }
        if (st != 0u) break;
        expand_chunk(toks, cnt);
        if (why == kEndOfBlock) break;
        if (why == kNeedInput) stage(ub.p & ~15u);
      }
      br.buf = ub.buf;
      br.n = ub.n;
      br.p = ub.p;
      if (st != 0u) break;
    }
    if (lane == 0 && 8ull * br.p - br.n > 8ull * len) st = kStBad;
    st = bcast32(st);
    if (st != 0u) break;
    e = bcast64(8ull * br.p - br.n);
    if (last || e >= target) break;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) res[r] = SplitResult{e, o, (last ? 1u : 0u) | (st << 8)};
}

// K8s-resolve: one 256-thread workgroup per split stream (stream index
// `sidx[b]`, its regions [first, first + count)).  status 0 = inflated and
// Adler-32 verified; 0xFF = not resolved here (the engine reruns the stream
// with hbx_k8_inflate).
extern "C" __global__ __launch_bounds__(256) void hbx_k8s_resolve(
    const InflateDesc* __restrict__ desc, const uint32_t* __restrict__ sidx, const uint32_t* __restrict__ sfirst,
    const uint32_t* __restrict__ scount, uint32_t nstreams, const SplitRegion* __restrict__ reg,
    const uint64_t* __restrict__ start, const SplitResult* __restrict__ res, const uint16_t* __restrict__ scratch,
    uint32_t* __restrict__ out_len, uint32_t* __restrict__ status) {
  using namespace hbxs;
  const uint32_t b = blockIdx.x;
  if (b >= nstreams) return;
  const uint32_t tid = threadIdx.x;
  const uint32_t i = sidx[b], first = sfirst[b], count = scount[b];
  const InflateDesc d = desc[i];
  const uint8_t* src = reinterpret_cast<const uint8_t*>(d.src);
  uint8_t* out = reinterpret_cast<uint8_t*>(d.dst);
  const uint64_t len = d.len, cap = d.cap;
  __shared__ uint32_t red[2][4];
  uint64_t pos = 0;          // output bytes written (uniform)
  uint32_t cur = 0;          // region (within the stream)
  bool ok = true, done = false;
  uint32_t a0 = 0u;          // this thread's Adler partial sums: sum x, sum pos * x
  uint64_t a1 = 0ull;
  uint64_t steps = 0;
  while (ok && !done) {
    const SplitResult rr = res[first + cur];
    const SplitRegion R = reg[first + cur];
    const uint32_t n = rr.nsym;
    if ((rr.flags >> 8) != 0u || pos + n > cap) {
      ok = false;
      break;
    }
    const uint16_t* sy = scratch + R.sym;
    // markers read the output of earlier regions: every store of theirs must
    // be complete, and their reads must miss the (non-coherent) L1
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    bool bad = false;
    for (uint32_t q = tid; q < n; q += 256u) {
      const uint32_t v = sy[q];
      uint32_t x;
      if (v & 0x8000u) {
        const int64_t at = (int64_t)pos - 32768 + (int64_t)(v & 0x7FFFu);
        if (at < 0) {
          bad = true;
          x = 0u;
        } else {
          const uint64_t ad = reinterpret_cast<uint64_t>(out) + (uint64_t)at;
          const uint32_t* w = reinterpret_cast<const uint32_t*>(ad & ~3ull);
          const uint32_t word = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          x = (word >> (8u * (uint32_t)(ad & 3u))) & 0xFFu;
        }
      } else {
        x = v & 0xFFu;
      }
      out[pos + q] = (uint8_t)x;
      a0 += x;
      a1 += (pos + q) * (uint64_t)x;
      if ((++steps & 0xFFFFull) == 0ull) {
        a0 %= kAdlerMod;
        a1 %= kAdlerMod;
      }
    }
    if (__syncthreads_or(bad)) {
      ok = false;
      break;
    }
    pos += n;
    if (rr.flags & 1u) {
      done = true;
      break;
    }
    // the next region of the chain starts exactly where this one ended
    uint32_t nx = cur + 1u;
    while (nx < count && start[first + nx] == kNoStart) nx++;
    if (nx >= count || start[first + nx] != rr.end_bit) {
      ok = false;
      break;
    }
    cur = nx;
  }
  // Adler-32 of the bytes written against the trailer after the final block
  uint32_t aa = a0 % kAdlerMod, bb = (uint32_t)(a1 % kAdlerMod);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    aa = (aa + (uint32_t)__shfl_xor((int)aa, off, 64)) % kAdlerMod;
    bb = (bb + (uint32_t)__shfl_xor((int)bb, off, 64)) % kAdlerMod;
  }
  if ((tid & 63u) == 0u) {
    red[0][tid >> 6] = aa;
    red[1][tid >> 6] = bb;
  }
  __syncthreads();
  if (tid == 0) {
    bool good = ok && done;
    if (good) {
      uint32_t A = 0u, B = 0u;
      for (int w = 0; w < 4; w++) {
        A = (A + red[0][w]) % kAdlerMod;
        B = (B + red[1][w]) % kAdlerMod;
      }
      const SplitResult rr = res[first + cur];
      const uint64_t q = (rr.end_bit + 7u) >> 3;
      if (q + 4u > len) {
        good = false;
      } else {
        const uint32_t want = ((uint32_t)src[q] << 24) | ((uint32_t)src[q + 1] << 16) |
                              ((uint32_t)src[q + 2] << 8) | (uint32_t)src[q + 3];
        const uint64_t om = pos % kAdlerMod;
        const uint32_t AA = (uint32_t)((1u + A) % kAdlerMod);
        const uint32_t BB = (uint32_t)((om + om * A + kAdlerMod - B) % kAdlerMod);
        good = ((BB << 16) | AA) == want;
      }
    }
    out_len[i] = good ? (uint32_t)pos : 0u;
    status[i] = good ? 0u : 0xFFu;
  }
}

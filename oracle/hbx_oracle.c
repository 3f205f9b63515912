/*
 * hbx_oracle.c — CPU ORACLE FOR THE ROLLSUM-SPLIT + BLOCK-ID PATH.
 *
 *   TEST INFRASTRUCTURE ONLY.  Nothing in the product (hashbox_amd/, the
 *   libhbxgpu C-ABI) links, loads or calls this file.  Only tests/,
 *   __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only
 *   as the checker / the timed CPU baseline ("kind": "port").
 *
 * It is a plain-C restatement of the reference algorithm:
 *
 *   - chunk driver      hashback/store.go:111-185  (storeFile loop)
 *   - split rule        hashback/store.go:129-166  (last max digest, ">=" at :160)
 *   - size constants    hashback/hashback.go:37-38 (MAX 8 MiB, MIN 64 KiB)
 *   - block id          pkg/core/block.go:39-43, 49-55, 96-111
 *                       BlockID = MD5(BE32(nlinks) || links || BE32(len) || data)
 *   - BE32 framing      pkg/core/utils.go:81-84
 *   - file chain block  hashback/hashback.go:156-170, store.go:187-196
 *   - MD5               Go crypto/md5 (block.go:14,99) == RFC 1321, written
 *                       here from the RFC; pinned by the HMAC-MD5 KATs of
 *                       pkg/core/core_test.go:23-30 and by Python hashlib.
 *
 * Third-party arithmetic: github.com/smtc/rollsum @ v0.0.0-20150721100732-
 * 39e98d252100 (hashback/go.mod:10, go.sum:7) is NOT present in the
 * container.  Its API shape (Init/Rollin/Rollout/Digest() uint32, called at
 * store.go:131-132,152,155,159) is the librsync rolling checksum; that
 * published algorithm is restated in the ONE isolated block marked
 * "ASSUMPTION A1" below.  Cut points are therefore
 * "parity: oracle-consistent, reference-unpinned" for the rollsum part;
 * block IDs and the split rule are pinned by source + MD5 KATs.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define HBXO_MIN_BLOCK ((uint64_t)65536)    /* hashback/hashback.go:38 */
#define HBXO_MAX_BLOCK ((uint64_t)8388608)  /* hashback/hashback.go:37 */

/* ------------------------------------------------------------------------ */
/* MD5 (RFC 1321).                                                          */
/* ------------------------------------------------------------------------ */

typedef struct {
    uint32_t h[4];
    uint64_t nbytes;
    uint8_t buf[64];
    uint32_t nbuf;
} hbxo_md5_t;

static const uint32_t MD5_T[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const uint8_t MD5_R[64] = {
    7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
    5, 9, 14, 20, 5, 9, 14, 20, 5, 9, 14, 20, 5, 9, 14, 20,
    4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
    6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static inline uint32_t rotl32(uint32_t x, unsigned s) { return (x << s) | (x >> (32 - s)); }

static void md5_compress(uint32_t h[4], const uint8_t *p) {
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
               ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) {
            f = (b & c) | (~b & d);
            g = i;
        } else if (i < 32) {
            f = (d & b) | (~d & c);
            g = (5 * i + 1) & 15;
        } else if (i < 48) {
            f = b ^ c ^ d;
            g = (3 * i + 5) & 15;
        } else {
            f = c ^ (b | ~d);
            g = (7 * i) & 15;
        }
        uint32_t t = d;
        d = c;
        c = b;
        b = b + rotl32(a + f + MD5_T[i] + m[g], MD5_R[i]);
        a = t;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

void hbxo_md5_init(hbxo_md5_t *s) {
    s->h[0] = 0x67452301;
    s->h[1] = 0xefcdab89;
    s->h[2] = 0x98badcfe;
    s->h[3] = 0x10325476;
    s->nbytes = 0;
    s->nbuf = 0;
}

void hbxo_md5_update(hbxo_md5_t *s, const uint8_t *p, uint64_t n) {
    s->nbytes += n;
    if (s->nbuf) {
        uint32_t take = 64 - s->nbuf;
        if (take > n) take = (uint32_t)n;
        memcpy(s->buf + s->nbuf, p, take);
        s->nbuf += take;
        p += take;
        n -= take;
        if (s->nbuf < 64) return;
        md5_compress(s->h, s->buf);
        s->nbuf = 0;
    }
    while (n >= 64) {
        md5_compress(s->h, p);
        p += 64;
        n -= 64;
    }
    if (n) {
        memcpy(s->buf, p, n);
        s->nbuf = (uint32_t)n;
    }
}

void hbxo_md5_final(hbxo_md5_t *s, uint8_t out[16]) {
    uint64_t bits = s->nbytes * 8;
    uint8_t pad[72];
    uint32_t padlen = (s->nbuf < 56) ? (56 - s->nbuf) : (120 - s->nbuf);
    memset(pad, 0, sizeof pad);
    pad[0] = 0x80;
    for (int i = 0; i < 8; i++) pad[padlen + i] = (uint8_t)(bits >> (8 * i));
    uint64_t keep = s->nbytes;
    hbxo_md5_update(s, pad, padlen + 8);
    s->nbytes = keep;
    for (int i = 0; i < 4; i++) {
        out[4 * i + 0] = (uint8_t)(s->h[i]);
        out[4 * i + 1] = (uint8_t)(s->h[i] >> 8);
        out[4 * i + 2] = (uint8_t)(s->h[i] >> 16);
        out[4 * i + 3] = (uint8_t)(s->h[i] >> 24);
    }
}

void hbxo_md5(const uint8_t *msg, uint64_t n, uint8_t out[16]) {
    hbxo_md5_t s;
    hbxo_md5_init(&s);
    hbxo_md5_update(&s, msg, n);
    hbxo_md5_final(&s, out);
}

/* pkg/core/utils.go:81-84 WriteUint32: big-endian. */
static void be32(uint8_t b[4], uint32_t v) {
    b[0] = (uint8_t)(v >> 24);
    b[1] = (uint8_t)(v >> 16);
    b[2] = (uint8_t)(v >> 8);
    b[3] = (uint8_t)v;
}

/* pkg/core/block.go:96-111 HashData (+ SerializeLinks block.go:49-55).
 * The DataType byte is NOT hashed (block.go:101).  Length is uint32. */
void hbxo_block_id(const uint8_t *links, uint32_t nlinks, const uint8_t *data, uint64_t len,
                   uint8_t out[16]) {
    hbxo_md5_t s;
    uint8_t b[4];
    hbxo_md5_init(&s);
    be32(b, nlinks);
    hbxo_md5_update(&s, b, 4);
    if (nlinks) hbxo_md5_update(&s, links, (uint64_t)nlinks * 16);
    be32(b, (uint32_t)len);
    hbxo_md5_update(&s, b, 4);
    hbxo_md5_update(&s, data, len);
    hbxo_md5_final(&s, out);
}

/* ------------------------------------------------------------------------ */
/* ASSUMPTION A1 — smtc/rollsum == librsync rollsum.         */
/* All three degrees of freedom that could change results live here:        */
/*   (i) digest packing order  HBXO_A1_PACK_S2_HIGH                          */
/*   (ii) weight direction      (Rollin adds s1 into s2: oldest byte weighs n)*/
/*   (iii) char offset parity   HBXO_A1_CHAR_OFFSET (31, odd)                */
/* ------------------------------------------------------------------------ */
#define HBXO_A1_CHAR_OFFSET 31u
#define HBXO_A1_PACK_S2_HIGH 1

typedef struct {
    uint64_t count, s1, s2;
} hbxo_rollsum_t;

static inline void rs_init(hbxo_rollsum_t *r) { r->count = r->s1 = r->s2 = 0; }
static inline void rs_rollin(hbxo_rollsum_t *r, uint8_t c) {
    r->s1 += (uint64_t)c + HBXO_A1_CHAR_OFFSET;
    r->s2 += r->s1;
    r->count++;
}
static inline void rs_rollout(hbxo_rollsum_t *r, uint8_t c) {
    r->s1 -= (uint64_t)c + HBXO_A1_CHAR_OFFSET;
    r->s2 -= r->count * ((uint64_t)c + HBXO_A1_CHAR_OFFSET);
    r->count--;
}
static inline uint32_t rs_digest(const hbxo_rollsum_t *r) {
#if HBXO_A1_PACK_S2_HIGH
    return (uint32_t)((r->s2 << 16) | (r->s1 & 0xffff));
#else
    return (uint32_t)((r->s1 << 16) | (r->s2 & 0xffff));
#endif
}
/* ---------------------------- end of A1 --------------------------------- */

/* Digest of one window (Init + n Rollins + Digest): exposed for tests. */
uint32_t hbxo_window_digest(const uint8_t *w, uint64_t n) {
    hbxo_rollsum_t r;
    rs_init(&r);
    for (uint64_t i = 0; i < n; i++) rs_rollin(&r, w[i]);
    return rs_digest(&r);
}

/* Split position of one fill buffer: a literal restatement of
 * hashback/store.go:129-166 (Rollout before Rollin once rollInPos >= MIN,
 * Digest after the Rollin once rollInPos >= MIN, ">=" keeps the LAST max). */
static uint64_t split_literal(const uint8_t *buf, uint64_t len) {
    uint64_t split = len; /* store.go:129 default: whole buffer */
    if (len > 2 * HBXO_MIN_BLOCK) { /* store.go:130 strictly greater */
        hbxo_rollsum_t r;
        rs_init(&r);
        uint32_t maxd = 0;
        uint64_t in = 0, out = 0;
        while (in < len) {
            if (in >= HBXO_MIN_BLOCK) {
                rs_rollout(&r, buf[out]);
                out++;
            }
            rs_rollin(&r, buf[in]);
            in++;
            if (in >= HBXO_MIN_BLOCK) {
                uint32_t d = rs_digest(&r);
                if (d >= maxd) {
                    maxd = d;
                    split = in;
                }
            }
        }
    }
    return split;
}

/* hashback/hashback.go:156-170 FileChainBlock.Serialize + store.go:187-188:
 * data = "fchn" || BE32(k) || sum(id_i || decryptkey_i(=0^16)); links = ids. */
void hbxo_chain_id(const uint8_t *ids, uint64_t k, uint8_t out[16]) {
    uint64_t dlen = 8 + 32 * k;
    uint8_t *data = (uint8_t *)malloc(dlen);
    be32(data, 0x6663686Eu);
    be32(data + 4, (uint32_t)k);
    for (uint64_t i = 0; i < k; i++) {
        memcpy(data + 8 + 32 * i, ids + 16 * i, 16);
        memset(data + 8 + 32 * i + 16, 0, 16);
    }
    hbxo_block_id(ids, (uint32_t)k, data, dlen, out);
    free(data);
}

/* storeFile (hashback/store.go:84-199) over an in-memory file.
 * Returns the number of chunks (or -1 if cap is too small).  cut_ends[i] is
 * the file offset where chunk i ends; ids[16*i..] its BlockID.  content_id /
 * content_type follow store.go:187-196 (2 = FileData, 3 = FileChain). */
int64_t hbxo_store_file(const uint8_t *data, uint64_t n, uint64_t *cut_ends, uint8_t *ids,
                        uint64_t cap, uint8_t content_id[16], int32_t *content_type) {
    uint64_t k = 0;
    uint64_t off = 0;
    while (off < n) {
        uint64_t left = n - off;
        uint64_t L = left < HBXO_MAX_BLOCK ? left : HBXO_MAX_BLOCK; /* store.go:116-120 */
        uint64_t split = split_literal(data + off, L);
        if (k >= cap) return -1;
        if (cut_ends) cut_ends[k] = off + split;
        if (ids) hbxo_block_id(NULL, 0, data + off, split, ids + 16 * k);
        k++;
        off += split;
    }
    if (content_id && ids) {
        if (k > 1) {
            hbxo_chain_id(ids, k, content_id);
            if (content_type) *content_type = 3; /* ContentTypeFileChain */
        } else if (k == 1) {
            memcpy(content_id, ids, 16);
            if (content_type) *content_type = 2; /* ContentTypeFileData */
        }
    }
    return (int64_t)k;
}

/* Closed form of the window digest at every position:
 * D[q] = digest of window data[q-MIN+1 .. q] with virtual zeros before the
 * file start, for q in [0, n).  Used to cross-check the literal loop and as
 * the reference for the device's per-position digest.  O(n). */
void hbxo_digest_all(const uint8_t *data, uint64_t n, uint32_t *D) {
    uint32_t s1 = 0, s2 = 0x8000u; /* virtual-zero prefix: s2 = 2^15 (offset 31 odd) */
    for (uint64_t q = 0; q < n; q++) {
        uint32_t out = (q >= HBXO_MIN_BLOCK) ? data[q - HBXO_MIN_BLOCK] : 0u;
        s1 = (s1 + data[q] - out) & 0xffffu;
        s2 = (s2 + s1) & 0xffffu;
        D[q] = (s2 << 16) | s1;
    }
}

/* Fast (closed-form) storeFile: same results as hbxo_store_file, O(n) digest
 * work instead of the reference's re-rolled windows.  Cross-check only. */
int64_t hbxo_store_file_fast(const uint8_t *data, uint64_t n, uint64_t *cut_ends, uint8_t *ids,
                             uint64_t cap, uint8_t content_id[16], int32_t *content_type) {
    uint32_t *D = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    hbxo_digest_all(data, n, D);
    uint64_t k = 0, off = 0;
    while (off < n) {
        uint64_t left = n - off;
        uint64_t L = left < HBXO_MAX_BLOCK ? left : HBXO_MAX_BLOCK;
        uint64_t split = L;
        if (L > 2 * HBXO_MIN_BLOCK) {
            uint32_t best = 0;
            for (uint64_t p = off + HBXO_MIN_BLOCK; p <= off + L; p++) {
                uint32_t d = D[p - 1];
                if (d >= best) {
                    best = d;
                    split = p - off;
                }
            }
        }
        if (k >= cap) {
            free(D);
            return -1;
        }
        if (cut_ends) cut_ends[k] = off + split;
        if (ids) hbxo_block_id(NULL, 0, data + off, split, ids + 16 * k);
        k++;
        off += split;
    }
    free(D);
    if (content_id && ids) {
        if (k > 1) {
            hbxo_chain_id(ids, k, content_id);
            if (content_type) *content_type = 3;
        } else if (k == 1) {
            memcpy(content_id, ids, 16);
            if (content_type) *content_type = 2;
        }
    }
    return (int64_t)k;
}

/* Multi-threaded batch driver for the CPU baseline: files are independent,
 * each handled by the literal single-goroutine loop above (the reference runs
 * one storeFile per goroutine).  Threads pull files from a
 * shared counter.  Outputs: per-file chunk counts; cut/id arrays laid out at
 * out_base[f] (caller-provided, each with per-file capacity). */
typedef struct {
    const uint8_t *const *datas;
    const uint64_t *lens;
    uint64_t nfiles;
    uint64_t *cut_ends;
    uint8_t *ids;
    const uint64_t *out_base;
    const uint64_t *caps;
    int64_t *counts;
    volatile uint64_t next;
    pthread_mutex_t mu;
} batch_job_t;

static void *batch_worker(void *arg) {
    batch_job_t *j = (batch_job_t *)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint64_t f = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (f >= j->nfiles) break;
        uint64_t b = j->out_base[f];
        j->counts[f] = hbxo_store_file(j->datas[f], j->lens[f], j->cut_ends + b, j->ids + 16 * b,
                                       j->caps[f], NULL, NULL);
    }
    return NULL;
}

int hbxo_store_batch_mt(const uint8_t *const *datas, const uint64_t *lens, uint64_t nfiles,
                        uint64_t *cut_ends, uint8_t *ids, const uint64_t *out_base,
                        const uint64_t *caps, int64_t *counts, int nthreads) {
    batch_job_t j;
    j.datas = datas;
    j.lens = lens;
    j.nfiles = nfiles;
    j.cut_ends = cut_ends;
    j.ids = ids;
    j.out_base = out_base;
    j.caps = caps;
    j.counts = counts;
    j.next = 0;
    pthread_mutex_init(&j.mu, NULL);
    if (nthreads < 1) nthreads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&j.mu);
    return 0;
}

/* HMAC-MD5 as pkg/core/core.go:51-69 (Hmac over a Byte128 key) and
 * DeepHmac core.go:72-80, so the KATs at pkg/core/core_test.go:23-30 can pin
 * this MD5 directly. */
void hbxo_hmac(const uint8_t *data, uint64_t n, const uint8_t key16[16], uint8_t out[16]) {
    uint8_t ipad[64], opad[64], inner[16];
    memset(ipad, 0, 64);
    memcpy(ipad, key16, 16);
    memcpy(opad, ipad, 64);
    for (int i = 0; i < 64; i++) {
        ipad[i] ^= 0x36;
        opad[i] ^= 0x5c;
    }
    hbxo_md5_t s;
    hbxo_md5_init(&s);
    hbxo_md5_update(&s, ipad, 64);
    hbxo_md5_update(&s, data, n);
    hbxo_md5_final(&s, inner);
    hbxo_md5_init(&s);
    hbxo_md5_update(&s, opad, 64);
    hbxo_md5_update(&s, inner, 16);
    hbxo_md5_final(&s, out);
}

void hbxo_deep_hmac(int depth, const uint8_t *data, uint64_t n, const uint8_t key16[16],
                    uint8_t out[16]) {
    uint8_t h[16];
    const uint8_t *d = data;
    uint64_t dn = n;
    for (int i = 0; i < depth; i++) {
        hbxo_hmac(d, dn, key16, h);
        d = h;
        dn = 16;
    }
    memcpy(out, h, 16);
}

/*
 * hbxgpu.h — C-ABI of the MI355X rollsum-split + block-ID engine
 * (libhbxgpu.so).  Drop-in for Hashback's per-file chunker and block hashing.
 *
 * Reference interfaces replaced (fredli74/hashbox; the reference has no FFI
 * seam for this path, so the seam is cut at storeFile — SURVEY.md §8b):
 *
 *   hbx_chunk_hash        hashback/store.go:111-185  storeFile's split loop
 *                         (store.go:129-166) + the per-chunk
 *                         Client.StoreData -> NewHashboxBlock -> HashData
 *                         (pkg/core/client.go:556-560, block.go:39-43, 96-111)
 *   hbx_chunk_hash_batch  the same, for many files at once (tree walk order
 *                         store.go:201-397 is the caller's business)
 *   hbx_chunk_hash_device the same, files already resident in device memory
 *   hbx_submit_device /   asynchronous, pipelined form: any number of batches
 *   hbx_wait              in flight per context, completed in FIFO order
 *   hbx_store_paths       storeFile(path) for many files on disk, end to end
 *   hbx_block_id          HashboxBlock.HashData for an arbitrary block with
 *                         links (pkg/core/block.go:96-111), e.g. the
 *                         FileChainBlock of store.go:187-188
 *   hbx_file_summary      entry.ContentType / entry.ContentBlockID written by
 *                         store.go:187-196
 *   hbx_verify_blocks     HashboxBlock.VerifyBlock (block.go:152-174), batched
 *   hbx_file_entry_*,     FileEntry / FileChainBlock / DirectoryBlock
 *   hbx_chain_block_*,    Serialize + Unserialize (hashback/hashback.go:80-214)
 *   hbx_directory_block_* and storeDir's block id (store.go:201-234)
 *   hbx_deflate_blocks    HashboxBlock.CompressData, zlib (block.go:133-184)
 *   hbx_inflate_blocks_device  UncompressData (block.go:113-131), on the device
 *   hbx_wire_*            ProtocolMessage framing of every message type
 *                         (pkg/core/protocol.go:184-264), block-store encoders
 *
 * Conventions
 *   - Every function returns an int status: 0 = OK, negative = error
 *     (HBX_ERR_*).  hbx_last_error(ctx) describes the last failure.  The
 *     library never aborts or exits (the Go wrapper turns a non-zero status
 *     into core.Abort, pkg/core/utils.go:22-37).
 *   - The caller owns every buffer passed in.  The library never frees caller
 *     memory and never keeps a caller pointer after the call returns, except
 *     between hbx_submit_device and the hbx_wait that completes the batch,
 *     where the device arena and the output arrays must stay valid (use
 *     hbx_alloc_pinned memory from cgo: cgo forbids C from retaining Go
 *     pointers).
 *   - One context = one GPU and its own HIP streams.  Calls on one context are
 *     serialised by an internal lock; use one context per GPU (or per
 *     goroutine) to run in parallel.
 *   - Block IDs are 16 raw MD5 bytes, exactly Go's core.Byte128 (core.go:26).
 *   - cut_ends[i] is the file offset where chunk i ends (exclusive); chunk i
 *     starts at cut_ends[i-1] (0 for i = 0).
 *   - Capacity: every chunk except the last is >= 64 KiB, so a file of len
 *     bytes has at most hbx_max_chunks(len) = len/65536 + 1 chunks.
 *   - Device inputs must be complete when the engine reads them: its HIP
 *     streams do not wait for the caller's streams.  Synchronize the producing
 *     stream first, or call hbx_after_stream(ctx, stream) before the submit
 *     (a GPU-side wait; the host does not block).
 */
#ifndef HBXGPU_H
#define HBXGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HBX_OK 0
#define HBX_ERR_ARG (-1)
#define HBX_ERR_HIP (-2)
#define HBX_ERR_CAPACITY (-3)
#define HBX_ERR_IO (-4)
#define HBX_ERR_NODEV (-5)
#define HBX_ERR_STATE (-6)

#define HBX_MIN_BLOCK_SIZE 65536u   /* hashback/hashback.go:38 */
#define HBX_MAX_BLOCK_SIZE 8388608u /* hashback/hashback.go:37 */
#define HBX_CONTENT_FILE_DATA 2     /* ContentTypeFileData,  store.go:193 */
#define HBX_CONTENT_FILE_CHAIN 3    /* ContentTypeFileChain, store.go:189 */
/* Device arenas must be readable this many bytes past the end of every file
 * (loads are 16-byte granular and bounds-checked, never fault, but the last
 * granule of a file may straddle its end). */
#define HBX_ARENA_SLACK 64u
#define HBX_ARENA_ALIGN 16u

typedef struct hbx_ctx hbx_ctx;

/* Per-file result beside the chunk list (store.go:187-196). */
typedef struct {
  uint8_t content_id[16]; /* entry.ContentBlockID */
  int32_t content_type;   /* 2 = FileData (1 chunk), 3 = FileChain, 0 = empty */
  uint32_t n_chunks;
} hbx_file_summary;

int hbx_version(void);
int hbx_device_count(int *n);
uint64_t hbx_max_chunks(uint64_t len);

int hbx_ctx_create(int device, hbx_ctx **out);
void hbx_ctx_destroy(hbx_ctx *ctx);
const char *hbx_last_error(const hbx_ctx *ctx);

/* One file in host memory (the storeFile drop-in).  ids must hold 16*cap
 * bytes; *n_chunks receives the chunk count. */
int hbx_chunk_hash(hbx_ctx *ctx, const uint8_t *data, uint64_t len, uint64_t *cut_ends,
                   uint8_t *ids, uint64_t cap, uint64_t *n_chunks);

/* Many files in host memory.  File f's chunks go to cut_ends[out_base[f] ..]
 * and ids[16*out_base[f] ..], at most caps[f] of them; summaries[f] gets the
 * count and the file content id. */
int hbx_chunk_hash_batch(hbx_ctx *ctx, uint64_t n_files, const uint8_t *const *datas,
                         const uint64_t *lens, uint64_t *cut_ends, uint8_t *ids,
                         const uint64_t *out_base, const uint64_t *caps,
                         hbx_file_summary *summaries);

/* Files already in device memory: file f is d_arena[file_offs[f] ..
 * +file_lens[f]).  file_offs must be multiples of HBX_ARENA_ALIGN and each
 * file must be followed by HBX_ARENA_SLACK readable bytes. */
int hbx_chunk_hash_device(hbx_ctx *ctx, const void *d_arena, uint64_t n_files,
                          const uint64_t *file_offs, const uint64_t *file_lens,
                          uint64_t *cut_ends, uint8_t *ids, const uint64_t *out_base,
                          const uint64_t *caps, hbx_file_summary *summaries);

/* Asynchronous device form: enqueue on the context's stream and return at
 * once.  Batches pipeline: the block-MD5 stage is time-sliced
 * (hbx_set_md5_slice), so the chunks of a new batch join the chains of the
 * batches still in flight instead of waiting behind their longest chunk.
 * hbx_wait completes the OLDEST pending batch and fills the output arrays
 * given at its submit (it first drains every chain in flight if that batch's
 * chains are not yet guaranteed hashed).  The synchronous calls
 * (hbx_chunk_hash*, hbx_store_paths) fail with HBX_ERR_STATE while batches
 * are pending. */
int hbx_submit_device(hbx_ctx *ctx, const void *d_arena, uint64_t n_files,
                      const uint64_t *file_offs, const uint64_t *file_lens, uint64_t *cut_ends,
                      uint8_t *ids, const uint64_t *out_base, const uint64_t *caps,
                      hbx_file_summary *summaries);
int hbx_wait(hbx_ctx *ctx);
/* Number of submitted batches not yet completed by hbx_wait. */
int hbx_pending(hbx_ctx *ctx);
/* Time slice of the block-MD5 stage: full 64-byte MD5 blocks each chain in
 * flight advances per launch (default 16384 = 1 MiB; 0 = unlimited, one
 * launch per batch); a chain takes the part short of a whole slice in its
 * first launch and whole slices after.  A submitted batch is complete after join lag (below)
 * + ceil(min(longest file, 8 MiB)/64 / blocks) - 1 further launches; results are
 * identical for every setting. */
int hbx_set_md5_slice(hbx_ctx *ctx, uint32_t blocks);
/* Reuse the input memory of the OLDEST pending batch: order the engine's
 * next input copies (hbx_memcpy_h2d_async) and submitted batches (chunking
 * and verify) after the MD5 launch that finishes that batch, with a GPU-side
 * wait, so they touch the memory only once the batch's last chain is hashed —
 * before the batch is collected with hbx_wait, and without blocking the
 * host.  A ring of device arenas then needs no slot for results still on
 * their way to the host.  If that batch's last launch has not been issued
 * yet, the chains in flight are drained first (correct, only slower).
 * The wait is enqueued lazily, just before the next engine-issued copy or
 * submit (it then sits after the next MD5 plan, off the scan loop), so ONLY
 * engine-issued work is ordered by this call.  A caller that writes the
 * memory itself (its own stream, kernel or copy) calls hbx_input_fence
 * first. */
int hbx_input_after_oldest(hbx_ctx *ctx);
/* Enqueue the wait of the latest hbx_input_after_oldest now: on the engine's
 * scan stream and, if `stream` (a hipStream_t) is not NULL, on that stream
 * too, so the caller's own writes into the old batch's memory are ordered
 * after the MD5 launch that finishes it.  Nothing is enqueued once the host
 * has seen that launch complete.  Never blocks the host. */
int hbx_input_fence(hbx_ctx *ctx, void *stream);
/* Optional: pre-size the pipeline for `batches` batches in flight of up to
 * `files` files and `bytes` bytes each.  The batch pool, the MD5 chain tables
 * and the slice summaries are allocated now, so the steady state never
 * allocates (growing a buffer the streams share drains both streams).  Fails
 * with HBX_ERR_STATE while batches are pending. */
int hbx_reserve(hbx_ctx *ctx, uint32_t batches, uint64_t files, uint64_t bytes);

/* Files on disk, end to end (storeFile over a list of paths, store.go:84-199
 * with the tree walk left to the caller): io_threads read batches of up to
 * batch_bytes straight into two pinned slots; each batch is copied into a
 * ring of device arenas and pipelined like hbx_submit_device, so reading
 * batch b+1 overlaps the copy of batch b and the hashing of every batch
 * still in flight.  lens[i] must be the file sizes (stat); a file that cannot be
 * read in full fails the call with HBX_ERR_IO.  Outputs as
 * hbx_chunk_hash_batch. */
int hbx_store_paths(hbx_ctx *ctx, uint64_t n_files, const char *const *paths,
                    const uint64_t *lens, uint64_t *cut_ends, uint8_t *ids,
                    const uint64_t *out_base, const uint64_t *caps, hbx_file_summary *summaries,
                    uint32_t io_threads, uint64_t batch_bytes);

/* Host seconds hbx_store_paths spent, cumulative per context: [0] reading
 * files into pinned memory, [1] waiting for batches to be collected (a device
 * arena's reuse, and the drain at the end of the call), [2] waiting for a
 * pinned slot's H2D copy.  reset != 0 zeroes them. */
int hbx_io_times(hbx_ctx *ctx, double s[3], int reset);
/* Host time of the slowest single call since the last reset, ms: [0] one H2D
 * copy call (hbx_memcpy_h2d_async and the disk path's copies), [1] one batch
 * submit (hbx_submit_device and the disk path's submits).  reset != 0 zeroes
 * them after reading.  No reference counterpart: diagnostics (the copy call
 * once held the host ~7 ms while the runtime created an SDMA engine's queue,
 * DESIGN.md §8). */
int hbx_host_call_max(hbx_ctx *ctx, double ms[2], int reset);

/* MD5(data) on the device: core.Hash (pkg/core/core.go:46-48), the primitive
 * under core.Hmac / DeepHmac (core.go:51-80). */
int hbx_md5(hbx_ctx *ctx, const uint8_t *data, uint64_t len, uint8_t out[16]);

/* MD5(BE32(n_links) || links || BE32(len) || data) on the device. */
int hbx_block_id(hbx_ctx *ctx, const uint8_t *links, uint32_t n_links, const uint8_t *data,
                 uint64_t len, uint8_t out[16]);

/* Batched HashboxBlock.HashData / VerifyBlock (pkg/core/block.go:96-111,
 * 152-174) for uncompressed blocks (BlockDataTypeRaw, or data already
 * inflated).  Block i's ID is MD5(BE32(n_links[i]) || links || BE32(lens[i])
 * || data), its links being the n_links[i] 16-byte IDs at
 * links[16*link_base[i] ..] (host memory; links, link_base and n_links may
 * be NULL when no block has links).  ids (16*n bytes, may be NULL) receives
 * the IDs.  With expect != NULL (16*n bytes), ok[i] (may be NULL) = 1 where
 * the ID equals expect[16*i ..], 0 elsewhere, and *n_bad (may be NULL)
 * counts the mismatches.  Callers in the reference: restore
 * (hashback/restore.go:52, 256), the server's write check
 * (server/server.go:182), verify -content (pkg/storagedb/integrity.go:117,
 * 282), show-block (util/commands.go:212).  Refused (HBX_ERR_STATE) while
 * batches are pending. */
int hbx_verify_blocks(hbx_ctx *ctx, uint64_t n, const uint8_t *const *datas, const uint64_t *lens,
                      const uint8_t *links, const uint64_t *link_base, const uint32_t *n_links,
                      uint8_t *ids, const uint8_t *expect, uint8_t *ok, uint64_t *n_bad);
/* The same for blocks in device memory: block i is d_arena[offs[i] ..
 * +lens[i]), followed by HBX_ARENA_SLACK readable bytes. */
int hbx_verify_blocks_device(hbx_ctx *ctx, const void *d_arena, uint64_t n, const uint64_t *offs,
                             const uint64_t *lens, const uint8_t *links, const uint64_t *link_base,
                             const uint32_t *n_links, uint8_t *ids, const uint8_t *expect,
                             uint8_t *ok, uint64_t *n_bad);

/* ---- Per-file and per-directory block formats ------------
 * hashback/hashback.go:80-214.  FileEntry is one directory entry; its
 * ContentBlockID is a chunk id (type 2), a FileChainBlock id (type 3, see
 * hbx_file_summary) or a DirectoryBlock id (type 1).  Strings are raw bytes
 * (core.String, pkg/core/core.go:95-109); integers big-endian
 * (pkg/core/utils.go:73-88); file_mode is Go's os.FileMode bit layout and
 * mod_time is UnixNano (store.go:243-251).  These functions are pure host
 * code and need no context. */
#define HBX_CONTENT_EMPTY 0     /* ContentTypeEmpty,     hashback.go:94 */
#define HBX_CONTENT_DIRECTORY 1 /* ContentTypeDirectory, hashback.go:95 */
#define HBX_CONTENT_SYMLINK 4   /* ContentTypeSymLink,   hashback.go:98 */
#define HBX_ERR_FORMAT (-7)     /* corrupted or truncated serialized block */

typedef struct {
  const char *name; /* FileName (not NUL-terminated) */
  uint32_t name_len;
  uint32_t file_mode;  /* FileMode */
  int64_t file_size;   /* FileSize */
  int64_t mod_time;    /* ModTime */
  uint8_t reference_id[16];
  uint8_t content_id[16];  /* written for types 1, 2, 3 */
  uint8_t decrypt_key[16]; /* written for type 2 */
  const char *link;        /* FileLink, written for type 4 */
  uint32_t link_len;
  uint8_t content_type; /* 0 empty, 1 dir, 2 file data, 3 file chain, 4 symlink */
  uint8_t pad[3];
} hbx_file_entry;

/* Serialized size of FileEntry.Serialize (hashback.go:113-132). */
uint64_t hbx_file_entry_size(const hbx_file_entry *e);
/* FileEntry.Serialize into out[0..cap); *n = bytes written.
 * HBX_ERR_CAPACITY if cap is too small (nothing useful written). */
int hbx_file_entry_serialize(const hbx_file_entry *e, uint8_t *out, uint64_t cap, uint64_t *n);
/* FileEntry.Unserialize (hashback.go:133-155) of in[0..len); *used = bytes
 * consumed.  name/link point into `in`.  HBX_ERR_FORMAT for a wrong magic
 * ("corrupted FileEntry") or a short buffer. */
int hbx_file_entry_parse(const uint8_t *in, uint64_t len, hbx_file_entry *e, uint64_t *used);

/* FileChainBlock.Serialize (hashback.go:162-170): "fchn", k, then k pairs
 * (id, decrypt key); keys may be NULL (all zero, as store.go:175-184 writes
 * them).  Size is 8 + 32k.  This is the block whose HashData with links =
 * ids is hbx_file_summary.content_id for type 3. */
int hbx_chain_block_serialize(const uint8_t *ids, const uint8_t *keys, uint32_t k, uint8_t *out,
                              uint64_t cap, uint64_t *n);
/* FileChainBlock.Unserialize (hashback.go:171-185): *k = chain length; ids
 * and keys (each 16*cap bytes, may be NULL) receive up to cap entries
 * (HBX_ERR_CAPACITY if *k > cap). */
int hbx_chain_block_parse(const uint8_t *in, uint64_t len, uint32_t *k, uint8_t *ids, uint8_t *keys,
                          uint32_t cap);

/* DirectoryBlock.Serialize (hashback.go:192-199) of n entries in the order
 * given (storeDir sorts by name, store.go:217).  links (16*n bytes, may be
 * NULL) receives storeDir's link list: the content_id of every entry of type
 * 1, 2 or 3, in order (store.go:221-228); *n_links its length.  Size:
 * hbx_directory_block_size. */
uint64_t hbx_directory_block_size(const hbx_file_entry *entries, uint32_t n);
int hbx_directory_block_serialize(const hbx_file_entry *entries, uint32_t n, uint8_t *out,
                                  uint64_t cap, uint64_t *n_out, uint8_t *links, uint32_t *n_links);
/* DirectoryBlock.Unserialize (hashback.go:200-214): *n = entry count;
 * entries[0..min(n, cap)) are filled (names/links point into `in`). */
int hbx_directory_block_parse(const uint8_t *in, uint64_t len, hbx_file_entry *entries, uint32_t cap,
                              uint32_t *n);

/* The IDs of many DirectoryBlocks at once, on the device: directory d holds
 * entries[entry_base[d] .. + n_entries[d]); ids[16*d ..] receives
 * NewHashboxBlock(dblk bytes, links).BlockID (store.go:230-231).  A tree's
 * directories are hashed level by level, deepest first, since a parent's
 * entry carries its child directory's id.  Refused (HBX_ERR_STATE) while
 * batches are pending. */
int hbx_directory_block_ids(hbx_ctx *ctx, uint32_t n_dirs, const hbx_file_entry *entries,
                            const uint64_t *entry_base, const uint32_t *n_entries, uint8_t *ids);

/* ---- zlib block compression ---------------------------------
 * HashboxBlock.CompressData for BlockDataTypeZlib (pkg/core/block.go:133-150,
 * 176-184; done by the client's workers before sending, client.go:249-258):
 * each block's data becomes one zlib stream (RFC 1950: 78 9C header, deflate
 * blocks, Adler-32).  Not byte-identical to Go's compress/zlib (the server
 * inflates and re-hashes, block.go:159-166; DataType is not hashed,
 * block.go:101) but every stream inflates to the block's data.  Each 32 KiB
 * segment is coded independently on the device (LZ77 within the segment +
 * fixed Huffman, or stored when that is not smaller), so any output is at
 * most hbx_deflate_bound(len) bytes. */
uint64_t hbx_deflate_bound(uint64_t len);
/* Blocks in device memory: block i = d_arena[offs[i] .. +lens[i]) (followed
 * by HBX_ARENA_SLACK readable bytes); its stream goes to d_out[out_offs[i] ..]
 * (out_caps[i] >= hbx_deflate_bound(lens[i]), else HBX_ERR_CAPACITY), its
 * length to out_lens[i] (host).  Synchronous.  Refused (HBX_ERR_STATE) while
 * batches are pending. */
int hbx_deflate_blocks_device(hbx_ctx *ctx, const void *d_arena, uint64_t n, const uint64_t *offs,
                              const uint64_t *lens, void *d_out, const uint64_t *out_offs,
                              const uint64_t *out_caps, uint64_t *out_lens);
/* The same for host blocks: datas[i] (lens[i] bytes) -> outs[i] (caps[i]
 * bytes), out_lens[i] = stream length. */
int hbx_deflate_blocks(hbx_ctx *ctx, uint64_t n, const uint8_t *const *datas, const uint64_t *lens,
                       uint8_t *const *outs, const uint64_t *caps, uint64_t *out_lens);

/* hbx_store_paths plus CompressData of every chunk on the device (the
 * client's send path: StoreData -> workers compress -> socket,
 * client.go:249-258).  sums is required.  Chunk i of file f (index
 * out_base[f] + i, like cut_ends) gets its zlib stream at zout[zoff[..]] with
 * length zlen[..]; file f's streams are packed from zout[zbase[f]], which
 * needs hbx_deflate_file_bound(lens[f]) bytes.
 * Device memory: each compression stage (two in flight) holds, besides its
 * output, 96 KiB of scratch per 32 KiB segment of the batch, about 3x the
 * batch's bytes (hbx_deflate.hip kSlot: the parse hand-off and the coded
 * image of every segment); hbx_deflate_blocks* hold the same per call.  Size
 * batch_bytes with that in mind. */
uint64_t hbx_deflate_file_bound(uint64_t len);
int hbx_store_paths_z(hbx_ctx *ctx, uint64_t n_files, const char *const *paths, const uint64_t *lens,
                      uint64_t *cut_ends, uint8_t *ids, const uint64_t *out_base, const uint64_t *caps,
                      hbx_file_summary *summaries, uint32_t io_threads, uint64_t batch_bytes,
                      uint8_t *zout, const uint64_t *zbase, uint64_t *zoff, uint64_t *zlen);

/* ---- wire protocol framing -----------------------------------
 * pkg/core/protocol.go: a message is u16 Num | u32 Type | its fields, big
 * endian (ProtocolMessage.Serialize, protocol.go:184-203).  Client types are
 * the lowercase constants; the server replies with Type & 0xDFDFDFDF
 * ("READ", "ACKN", "WRIT", "ERRS").  The StoreBlock exchange
 * (client.go:563-584, server.go:160-202): allo(id) -> READ(id) -> writ(block)
 * -> ACKN(id), or allo(id) -> ACKN(id) when the server has the block.  The
 * encoders cover that exchange; the parser frames every message type
 * protocol.go:204-264 knows.  Pure host code, no context. */
#define HBX_MSG_OLD_GREETING 0x686F6C61u /* "hola" */
#define HBX_MSG_GREETING 0x68616C6Fu    /* "halo" */
#define HBX_MSG_AUTHENTICATE 0x61757468u /* "auth" */
#define HBX_MSG_GOODBYE 0x71756974u     /* "quit" */
#define HBX_MSG_ACCOUNT_INFO 0x696E666Fu /* "info" */
#define HBX_MSG_ADD_DATASET_STATE 0x61646473u /* "adds" */
#define HBX_MSG_LIST_DATASET 0x6C697374u /* "list" */
#define HBX_MSG_REMOVE_DATASET_STATE 0x64656C73u /* "dels" */
#define HBX_MSG_ALLOCATE 0x616C6C6Fu    /* "allo" */
#define HBX_MSG_READ 0x72656164u        /* "read" */
#define HBX_MSG_WRITE 0x77726974u       /* "writ" */
#define HBX_MSG_ACKNOWLEDGE 0x61636B6Eu /* "ackn" */
#define HBX_MSG_ERROR 0x65727273u       /* "errs" (sent as "ERRS") */
#define HBX_SERVER_MASK 0xDFDFDFDFu
#define HBX_BLOCK_DATA_RAW 0xFFu  /* BlockDataTypeRaw,  block.go:21 */
#define HBX_BLOCK_DATA_ZLIB 0x01u /* BlockDataTypeZlib, block.go:22 */

typedef struct {
  uint16_t num;
  uint32_t type;
  uint8_t id[16];         /* allo/ACKN/read/READ/writ/WRIT: BlockID; HALO: nonce */
  uint32_t n_links;       /* writ/WRIT */
  const uint8_t *links;   /* writ/WRIT: into the input */
  uint8_t data_type;      /* writ/WRIT */
  uint32_t data_len;      /* writ/WRIT data; ERRS text; halo: version; others: payload bytes */
  const uint8_t *data;    /* writ/WRIT data, ERRS text, other payloads (after the 6-byte header): into the input */
  uint64_t header_len;    /* bytes before the data */
  uint64_t total_len;     /* bytes of the whole message */
} hbx_wire_msg;

/* allo / read (client) or ACKN / READ (server, pass type & HBX_SERVER_MASK):
 * 22 bytes. */
int hbx_wire_encode_id(uint16_t num, uint32_t type, const uint8_t id[16], uint8_t out[22]);
/* writ / WRIT up to (not including) the data: 31 + 16*n_links bytes; the
 * data_len bytes of block data follow on the wire as they are (for
 * BlockDataTypeZlib: the zlib stream, block.go:56-69). */
int hbx_wire_encode_block_header(uint16_t num, uint32_t type, const uint8_t id[16], const uint8_t *links,
                                 uint32_t n_links, uint8_t data_type, uint32_t data_len, uint8_t *out,
                                 uint64_t cap, uint64_t *n);
/* Parse one message at in[0..len) (ProtocolMessage.Unserialize,
 * protocol.go:204-264): HBX_OK, HBX_ERR_CAPACITY if the message is not
 * complete yet (msg->total_len is set once its header is), HBX_ERR_FORMAT for
 * an unknown type. */
int hbx_wire_parse(const uint8_t *in, uint64_t len, hbx_wire_msg *msg);

/* Pipelined VerifyBlock: the same inputs and outputs as
 * hbx_verify_blocks_device, enqueued like hbx_submit_device and completed by
 * hbx_wait in FIFO order with the chunking batches.  Each block's link prefix
 * is hashed first; the rest of its message joins the time-sliced MD5 chains
 * (hbx_set_md5_slice), so a bulk verification streams like the chunking path
 * instead of waiting on one launch's longest block.  ids, expect, ok and
 * n_bad must stay valid until the hbx_wait that completes the batch; links
 * are copied at submit. */
int hbx_verify_submit_device(hbx_ctx *ctx, const void *d_arena, uint64_t n, const uint64_t *offs,
                             const uint64_t *lens, const uint8_t *links, const uint64_t *link_base,
                             const uint32_t *n_links, uint8_t *ids, const uint8_t *expect,
                             uint8_t *ok, uint64_t *n_bad);

/* HashboxBlock.UncompressData for zlib blocks (pkg/core/block.go:113-131,
 * 186-201), many streams at once on the device: stream i =
 * d_in[in_offs[i] .. +in_lens[i]) inflates into d_out[out_offs[i] ..] (at most
 * out_caps[i] bytes); out_lens[i] (host) = inflated bytes, status[i] (host) =
 * 0, or 1 bad header / Adler-32, 2 truncated input, 3 output capacity,
 * 4 invalid code, 5 distance too far back, 6 bad stored length.  Any RFC
 * 1950 stream (Go's compress/zlib, K7's).  A corrupt stream only sets its
 * status.  Then hbx_verify_blocks_device / hbx_verify_submit_device on the
 * output is VerifyBlock of compressed blocks (block.go:152-166).
 * Synchronous; refused (HBX_ERR_STATE) while batches are pending. */
int hbx_inflate_blocks_device(hbx_ctx *ctx, const void *d_in, uint64_t n, const uint64_t *in_offs,
                              const uint64_t *in_lens, void *d_out, const uint64_t *out_offs,
                              const uint64_t *out_caps, uint64_t *out_lens, uint32_t *status);

/* hbx_store_paths_z with a callback per collected batch: ready(user, first,
 * count) runs as soon as files [first, first+count) have their cut_ends, ids,
 * summaries and zlib streams written, so a sender can put those blocks on the
 * wire while later batches are still read and hashed.  The calls come from
 * an engine worker thread (the one that unpacked the batch's compressed
 * streams), one at a time and in file order, all before this function
 * returns.  It must return quickly and must not call into the same context. */
typedef void (*hbx_batch_ready_fn)(void *user, uint64_t first_file, uint64_t n_files);
int hbx_store_paths_zcb(hbx_ctx *ctx, uint64_t n_files, const char *const *paths, const uint64_t *lens,
                        uint64_t *cut_ends, uint8_t *ids, const uint64_t *out_base, const uint64_t *caps,
                        hbx_file_summary *summaries, uint32_t io_threads, uint64_t batch_bytes,
                        uint8_t *zout, const uint64_t *zbase, uint64_t *zoff, uint64_t *zlen,
                        hbx_batch_ready_fn ready, void *user);

/* hbx_store_paths* with per-file outcomes (replaces the error handling of
 * storeFile/storePath/storeDir, hashback/store.go:85-94, 101-103, 221-224,
 * 356-359).  status (n_files int32, required) receives 0 for a file stored, or
 * the errno of a file the reference skips without stopping the tree walk:
 *   - open() failed (os.Open, store.go:101-103: storeDir logs "Skipping
 *     (ERROR)" and goes on with the next entry, :221-224);
 *   - a read failed with EBADF (minorPathError, hashback_unix.go:57-63:
 *     storePath keeps the previous backup's entry, store.go:356-359).
 * Such a file gets no chunks (summary n_chunks 0, content type 0); every other
 * file of its batch is stored as usual.  Any other read failure (an I/O error,
 * a file shorter than lens[i]) is what storeFile panics on (CopyNOrPanic,
 * pkg/core/utils.go:95-99): the call fails with HBX_ERR_IO and the path in
 * hbx_last_error, as hbx_store_paths does for every failure.  zout, zbase,
 * zoff, zlen all NULL: no compression (hbx_store_paths); else as
 * hbx_store_paths_zcb (ready may be NULL: hbx_store_paths_z). */
int hbx_store_paths_status(hbx_ctx *ctx, uint64_t n_files, const char *const *paths, const uint64_t *lens,
                           uint64_t *cut_ends, uint8_t *ids, const uint64_t *out_base, const uint64_t *caps,
                           hbx_file_summary *summaries, int32_t *status, uint32_t io_threads,
                           uint64_t batch_bytes, uint8_t *zout, const uint64_t *zbase, uint64_t *zoff,
                           uint64_t *zlen, hbx_batch_ready_fn ready, void *user);

/* Device arena helpers (allocations include HBX_ARENA_SLACK). */
int hbx_arena_alloc(hbx_ctx *ctx, uint64_t bytes, void **d_ptr);
int hbx_arena_free(hbx_ctx *ctx, void *d_ptr);
int hbx_memcpy_h2d(hbx_ctx *ctx, void *d_dst, const void *h_src, uint64_t bytes);
/* Enqueue an H2D copy on the context's stream and return at once: a
 * following hbx_submit_device on the same context runs after it.  h_src
 * should be hbx_alloc_pinned memory (pageable memory makes the copy
 * synchronous).  Use two contexts to overlap the next batch's copy with the
 * current batch's kernels. */
int hbx_memcpy_h2d_async(hbx_ctx *ctx, void *d_dst, const void *h_src, uint64_t bytes);
/* Order the context's next device work after everything enqueued so far on
 * `stream` (a hipStream_t of the same device, e.g. the stream that filled an
 * arena; NULL = the null stream).  The dependency is on the GPU (an event the
 * context's streams wait for): the host never blocks, so a caller can keep
 * submitting batches ahead of the device.  For the null stream and a blocking
 * scan stream (the default) the legacy default-stream ordering already holds
 * and nothing is recorded.  No reference counterpart: Go callers hand over
 * host buffers. */
int hbx_after_stream(hbx_ctx *ctx, void *stream);
int hbx_alloc_pinned(uint64_t bytes, void **out);
int hbx_free_pinned(void *p);

/* The context's effective pipeline knobs as one JSON object (NUL-terminated,
 * at most cap bytes): slice, join lag, K1 tile and run, K3 waves and placement,
 * and whether the HBX_* A/B environment switches were honoured (ab_env: they
 * are read only when HBX_AB=1).  No reference counterpart: diagnostics. */
int hbx_knobs(hbx_ctx *ctx, char *out, uint64_t cap);

/* Device time (ms) of the last completed batch per stage:
 * [0] K1 window-digest scan, [1] K2 cut chain, [2] K2 end -> results ready
 * (the batch's share of the pipelined MD5 launches, K4 and the copy),
 * [3] 0, [4] whole batch.  For a synchronous call [2] is the plan and K3
 * and [3] is K4 + the result copy. */
int hbx_stage_times(hbx_ctx *ctx, float ms[5]);
/* Cumulative device time (ms) and launch count per kernel since the context
 * was created (or last reset), for completed launches (K3 launches are timed
 * on the device and counted once known complete: after the wait that
 * collects a batch they finished, or once the hash stream is idle):
 * [0] K1 scan, [1] K2 cut chain, [2] K2c chain plan, [3] K3 block MD5,
 * [4] K4 content id.  reset != 0 zeroes the totals after reading. */
int hbx_stage_totals(hbx_ctx *ctx, double ms[5], uint64_t launches[5], int reset);
/* Diagnostics: turn the per-wave K3 records below on (on != 0) or off.
 * Changes no result and no other knob.  Fails with HBX_ERR_STATE while
 * batches are pending. */
int hbx_set_k3_probe(hbx_ctx *ctx, int on);
/* Diagnostics: with the probe on (hbx_set_k3_probe),
 * every K3 launch records per wave {start, end of its start-up (first
 * group's loads and prologue block) | XCC id << 56, end, R | max count << 16
 * | HW_ID << 32, s_memtime (shader cycles) at the start and the end of the
 * first group's cooperative phase, s_memrealtime at its end, the blocks of
 * each chain it hashed (R - 1) | the polls (s_sleep 1 each) in which the wave
 * found its producer's next stage not yet written, over the launch, << 32}
 * (times in s_memrealtime ticks, 100 MHz; R and
 * the count saturate at 65535; the last four are 0 for a wave whose first
 * group took the lane path).  Copies the latest launch's records (8 x u64 per
 * wave, up to max_waves) after the hash stream drains; *n_waves = waves per
 * launch. */
int hbx_k3_wave_times(hbx_ctx *ctx, uint64_t *out, uint32_t max_waves, uint32_t *n_waves);
/* Tile length of K1 in 64 KiB iterations, 1..1024; 0 (the default) sizes
 * tiles per batch: about two per CU, 16..256 iterations (1-16 MiB). */
int hbx_set_tile_iters(hbx_ctx *ctx, uint32_t iters);
/* Pipeline join lag, 1..4 (default 1): a batch's chains join the block-MD5
 * launch issued `lag` submits after it, so its cut stage (K1 scan + K2 cut
 * chain) has `lag` pipeline steps to finish before the hash stage needs it.
 * Lag 2 suits small batches, whose scan is latency- rather than
 * throughput-bound.  Results are identical for every setting; a batch is
 * complete `lag` - 1 launches later.  Fails with HBX_ERR_STATE while batches
 * are pending. */
int hbx_set_join_lag(hbx_ctx *ctx, uint32_t lag);
/* K3 period, 1..8 (default 1): one block-MD5 launch every `period` submits,
 * advancing every chain by `period` x the slice (hbx_set_md5_slice) and
 * joining every batch that is `lag` or more submits old (up to 8).  Each
 * launch has a fixed start-up and a tail (its slowest CU); a period > 1 pays
 * them once per `period` steps, which pays off for small batches (a rank's
 * 1 GiB share of configs[2] at N = 8).  Results are identical for every
 * setting; a batch completes up to `period` - 1 submits later.  Fails with
 * HBX_ERR_STATE while batches are pending. */
int hbx_set_k3_period(hbx_ctx *ctx, uint32_t period);

/* ---- Pipeline operating point ---------------------------------------------
 * Hashback calls storeFile once per file from its tree walk
 * (hashback/store.go:356 -> :84); a caller that batches those files for
 * hbx_submit_device reaches the engine's measured rate only with the
 * schedule below: R batches resident in device memory,
 * each MD5 launch advancing every chain by the slice, a join lag of 2, a
 * lead of 2 (3 below 64 files per batch) and, below 32 files per batch, one MD5
 * launch every 4 submits.
 * hbx_plan_pipeline computes that schedule (bench.py runs exactly this plan)
 * and hbx_apply_plan sets it on a context.  Request fields <= 0 (md5_slice:
 * < 0) are "auto"; a positive value overrides that knob. */
#define HBX_PLAN_HOST_INPUT 1u /* each batch is copied in from host memory per step: shallow pipeline */
#define HBX_PLAN_ARENA_SLACK (64ull << 20) /* planned per resident arena beyond its bytes (allocator rounding) */
typedef struct {
  uint64_t n_files;          /* files per batch on this device */
  uint64_t arena_bytes;      /* one batch's arena: last offset + last length + HBX_ARENA_SLACK (or more) */
  uint64_t longest_file;     /* bytes of the batch's longest file (its longest MD5 chain: min(this, 8 MiB)) */
  uint64_t free_bytes;       /* device memory to plan for; 0 = the context's device, free now */
  double hbm_frac;           /* share of free_bytes for resident arenas (<= 0: 0.95) */
  uint32_t ranks_per_device; /* processes sharing the device's memory (0: 1) */
  uint32_t steps;            /* submits the caller runs between drains (0: open-ended); an auto
                                period divides it */
  int32_t arenas;            /* resident batches R (<= 0: as many as hbm_frac of free_bytes holds) */
  int32_t md5_slice;         /* blocks per chain per submit (< 0: sized from R; 0: unlimited) */
  int32_t join_lag;          /* 1..4 (<= 0: 2) */
  int32_t lead;              /* steps an arena stays resident beyond its batch's launches (< 0: the join lag
                                at 64 or more files per batch with device input, else lag + 1) */
  int32_t k3_period;         /* 1..8 (<= 0: 4, or 2 if 4 does not divide steps, below 32 files; else 1) */
  uint32_t flags;            /* HBX_PLAN_HOST_INPUT */
} hbx_plan_request;
typedef struct {
  uint32_t resident;           /* R: batches in flight, one device arena each */
  uint32_t md5_slice;          /* for hbx_set_md5_slice (blocks per chain per submit; 0 = unlimited) */
  uint32_t join_lag;           /* for hbx_set_join_lag */
  uint32_t lead;               /* the arena of batch j is refilled for batch j + R (hbx_input_after_oldest) */
  uint32_t k3_period;          /* for hbx_set_k3_period */
  uint32_t launches_per_batch; /* MD5 launches a batch's longest chain needs */
  uint64_t hbm_bytes;          /* R x (arena_bytes + HBX_PLAN_ARENA_SLACK) */
} hbx_pipeline_plan;
/* Fill *plan from *req.  ctx may be NULL when req->free_bytes > 0 (pure
 * host arithmetic, no device call).  HBX_ERR_ARG for an impossible request
 * (no files, a knob out of range, or R too small for the launches a batch
 * needs: then hbx_last_error(ctx) says which; with ctx NULL,
 * hbx_last_error(NULL) describes the calling thread's last such failure). */
int hbx_plan_pipeline(hbx_ctx *ctx, const hbx_plan_request *req, hbx_pipeline_plan *plan);
/* Set the plan's slice, join lag and period on ctx and reserve R + 2 batches
 * of up to `files` files and `bytes` bytes (hbx_reserve).  The caller keeps R
 * arenas and, from the (R+1)-th submit on, calls hbx_input_after_oldest
 * before refilling the oldest one.  HBX_ERR_STATE while batches are pending. */
int hbx_apply_plan(hbx_ctx *ctx, const hbx_pipeline_plan *plan, uint64_t files, uint64_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* HBXGPU_H */

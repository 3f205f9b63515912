// hbx_formats.h — Hashback's per-file and per-directory block formats
// (SURVEY §8f1), host side of libhbxgpu.  Byte layouts follow
// hashback/hashback.go:80-214 with the big-endian helpers of
// pkg/core/utils.go:73-88 and core.String (pkg/core/core.go:95-109):
//
//   FileEntry       "fent" | u32 len(name) name | i64 size | u32 mode |
//                   i64 mtime | 16 reference id | u8 type |
//                   [16 content id if type 1,2,3] [16 decrypt key if type 2]
//                   [u32 len(link) link if type 4]        (hashback.go:113-132)
//   FileChainBlock  "fchn" | u32 k | k x (16 id | 16 decrypt key)
//                                                         (hashback.go:162-170)
//   DirectoryBlock  "dblk" | u32 n | n x FileEntry        (hashback.go:192-199)
//
// The parsers are the Unserialize methods (hashback.go:133-155, 171-185,
// 200-214): a wrong magic is "corrupted <type>", a short buffer is an error
// (the reference panics in io.ReadFull, pkg/core/utils.go:38-43).
// Parsed names and links point into the input buffer (no allocation).
#pragma once

#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/hbxgpu.h"

namespace hbxfmt {

constexpr uint32_t kMagicEntry = 0x66656E74u;  // "fent"
constexpr uint32_t kMagicChain = 0x6663686Eu;  // "fchn"
constexpr uint32_t kMagicDir = 0x64626C6Bu;    // "dblk"

// FileEntry.HasContentBlockID / HasDecryptKey / HasFileLink (hashback.go:100-108)
inline bool has_content(uint8_t t) { return t == 1 || t == 2 || t == 3; }
inline bool has_key(uint8_t t) { return t == 2; }
inline bool has_link(uint8_t t) { return t == 4; }

inline uint64_t entry_size(const hbx_file_entry& e) {
  uint64_t n = 4 + 4 + (uint64_t)e.name_len + 8 + 4 + 8 + 16 + 1;
  if (has_content(e.content_type)) n += 16;
  if (has_key(e.content_type)) n += 16;
  if (has_link(e.content_type)) n += 4 + (uint64_t)e.link_len;
  return n;
}

// Bounded big-endian writer; `ok` drops to false on overflow and stays so.
struct Writer {
  uint8_t* p;
  uint64_t cap, n = 0;
  bool ok = true;
  void bytes(const void* src, uint64_t len) {
    if (!ok || len > cap - n) {
      ok = false;
      return;
    }
    if (len) std::memcpy(p + n, src, len);
    n += len;
  }
  void u8(uint8_t v) { bytes(&v, 1); }
  void u32(uint32_t v) {
    const uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
    bytes(b, 4);
  }
  void i64(int64_t s) {
    const uint64_t v = (uint64_t)s;
    uint8_t b[8];
    for (int i = 0; i < 8; i++) b[i] = (uint8_t)(v >> (56 - 8 * i));
    bytes(b, 8);
  }
};

struct Reader {
  const uint8_t* p;
  uint64_t len, n = 0;
  bool ok = true;
  const uint8_t* take(uint64_t k) {
    if (!ok || k > len - n) {
      ok = false;
      return nullptr;
    }
    const uint8_t* r = p + n;
    n += k;
    return r;
  }
  uint8_t u8() {
    const uint8_t* b = take(1);
    return b ? b[0] : 0;
  }
  uint32_t u32() {
    const uint8_t* b = take(4);
    return b ? ((uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]) : 0u;
  }
  int64_t i64() {
    const uint8_t* b = take(8);
    uint64_t v = 0;
    if (b)
      for (int i = 0; i < 8; i++) v = v << 8 | b[i];
    return (int64_t)v;
  }
  void id(uint8_t out[16]) {
    const uint8_t* b = take(16);
    if (b)
      std::memcpy(out, b, 16);
    else
      std::memset(out, 0, 16);
  }
};

inline void write_entry(Writer& w, const hbx_file_entry& e) {
  w.u32(kMagicEntry);
  w.u32(e.name_len);
  w.bytes(e.name, e.name_len);
  w.i64(e.file_size);
  w.u32(e.file_mode);
  w.i64(e.mod_time);
  w.bytes(e.reference_id, 16);
  w.u8(e.content_type);
  if (has_content(e.content_type)) w.bytes(e.content_id, 16);
  if (has_key(e.content_type)) w.bytes(e.decrypt_key, 16);
  if (has_link(e.content_type)) {
    w.u32(e.link_len);
    w.bytes(e.link, e.link_len);
  }
}

// Returns "" on success, else the error text.
inline std::string read_entry(Reader& r, hbx_file_entry& e) {
  std::memset(&e, 0, sizeof(e));
  const uint32_t magic = r.u32();
  if (!r.ok) return "truncated FileEntry";
  if (magic != kMagicEntry) return "corrupted FileEntry";
  e.name_len = r.u32();
  e.name = reinterpret_cast<const char*>(r.take(e.name_len));
  e.file_size = r.i64();
  e.file_mode = r.u32();
  e.mod_time = r.i64();
  r.id(e.reference_id);
  e.content_type = r.u8();
  if (has_content(e.content_type)) r.id(e.content_id);
  if (has_key(e.content_type)) r.id(e.decrypt_key);
  if (has_link(e.content_type)) {
    e.link_len = r.u32();
    e.link = reinterpret_cast<const char*>(r.take(e.link_len));
  }
  return r.ok ? std::string() : std::string("truncated FileEntry");
}

inline uint64_t chain_size(uint32_t k) { return 8ull + 32ull * k; }

inline void write_chain(Writer& w, const uint8_t* ids, const uint8_t* keys, uint32_t k) {
  static const uint8_t zero[16] = {0};
  w.u32(kMagicChain);
  w.u32(k);
  for (uint32_t i = 0; i < k; i++) {
    w.bytes(ids + 16ull * i, 16);
    w.bytes(keys ? keys + 16ull * i : zero, 16);
  }
}

inline uint64_t dir_size(const hbx_file_entry* es, uint32_t n) {
  uint64_t s = 8;
  for (uint32_t i = 0; i < n; i++) s += entry_size(es[i]);
  return s;
}

// DirectoryBlock bytes plus storeDir's links: the ContentBlockIDs of the
// entries that have one, in directory order (store.go:221-228).
inline uint32_t write_dir(Writer& w, const hbx_file_entry* es, uint32_t n, uint8_t* links) {
  w.u32(kMagicDir);
  w.u32(n);
  uint32_t nl = 0;
  for (uint32_t i = 0; i < n; i++) {
    write_entry(w, es[i]);
    if (has_content(es[i].content_type)) {
      if (links) std::memcpy(links + 16ull * nl, es[i].content_id, 16);
      nl++;
    }
  }
  return nl;
}

}  // namespace hbxfmt

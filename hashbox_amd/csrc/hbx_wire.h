// hbx_wire.h — framing of the Hashbox wire protocol, host
// side of libhbxgpu.  pkg/core/protocol.go:
//
//   ProtocolMessage  u16 Num | u32 Type | fields in declaration order
//                    (Serialize, protocol.go:184-203); client types are the
//                    lowercase constants, server replies the same & 0xDFDFDFDF
//                    (protocol.go:37-70); Unserialize's type switch
//                    (protocol.go:204-264) decides which fields follow.
//   Block store (the hot path's exchange, client.go:563-584, server.go:160-202):
//     allo / ACKN / read / READ   + BlockID (16)             (protocol.go:100-131)
//     writ / WRIT      + HashboxBlock.Serialize (block.go:56-69):
//                      BlockID | u32 #links | links | u8 DataType | u32 len | data
//   Session:  halo + u32 Version;  HALO + SessionNonce (16);  hola, quit,
//             QUIT, AUTH, ADDS, DELS: nothing;  auth + 2 x Byte128;
//             ERRS + String (u32 len | bytes, core.go:95-109)
//   Account / dataset (core.go:111-228):
//     info + Byte128;  INFO + DatasetArray (u32 n | n x {String, i64, Byte128})
//     list + Byte128 + String;  LIST + DatasetStateArray (u32 n | n x {u8 flags,
//          StateID, BlockID, i64 Size, i64 UniqueSize}) + Byte128
//     adds + Byte128 + String + DatasetState (48);  dels + Byte128 + String + Byte128
//
// Everything big-endian (pkg/core/utils.go:73-88).  The parser frames any of
// these (total_len) and exposes the block-store fields; for the other
// messages `data`/`data_len` is the payload after the 6-byte header.
#pragma once

#include <cstdint>
#include <cstring>

#include "../../include/hbxgpu.h"
#include "hbx_formats.h"

namespace hbxwire {

constexpr uint32_t kServerMask = 0xDFDFDFDFu;  // protocol.go:67
constexpr uint32_t S(uint32_t t) { return t & kServerMask; }

inline bool is_id_msg(uint32_t t) {
  return t == HBX_MSG_ALLOCATE || t == HBX_MSG_READ || t == S(HBX_MSG_ALLOCATE) || t == S(HBX_MSG_READ) ||
         t == S(HBX_MSG_ACKNOWLEDGE);
}
inline bool is_block_msg(uint32_t t) { return t == HBX_MSG_WRITE || t == S(HBX_MSG_WRITE); }

// Cursor over the input that only counts: a field past the end leaves ok
// false (the message is incomplete, never an error).
struct Skip {
  const uint8_t* p;
  uint64_t len, n = 0;
  bool ok = true;
  void bytes(uint64_t k) {
    if (ok && len - n >= k) n += k;
    else ok = false;
  }
  uint32_t u32() {
    if (!ok || len - n < 4) {
      ok = false;
      return 0;
    }
    const uint8_t* q = p + n;
    n += 4;
    return (uint32_t)q[0] << 24 | (uint32_t)q[1] << 16 | (uint32_t)q[2] << 8 | q[3];
  }
  void string() { bytes(u32()); }
};

// Payload bytes of a non-block message after the 6-byte header, walked per
// its type.  Returns false for a type Unserialize does not know.
inline bool walk_payload(uint32_t t, Skip& k) {
  switch (t) {
    case HBX_MSG_OLD_GREETING: case HBX_MSG_GOODBYE: case S(HBX_MSG_GOODBYE): case S(HBX_MSG_AUTHENTICATE):
    case S(HBX_MSG_ADD_DATASET_STATE): case S(HBX_MSG_REMOVE_DATASET_STATE):
      return true;
    case HBX_MSG_GREETING: k.bytes(4); return true;
    case S(HBX_MSG_GREETING): case HBX_MSG_ACCOUNT_INFO: k.bytes(16); return true;
    case HBX_MSG_AUTHENTICATE: k.bytes(32); return true;
    case S(HBX_MSG_ERROR): k.string(); return true;
    case S(HBX_MSG_ACCOUNT_INFO): {  // DatasetArray
      const uint32_t n = k.u32();
      for (uint32_t i = 0; i < n && k.ok; i++) {
        k.string();
        k.bytes(8 + 16);
      }
      return true;
    }
    case HBX_MSG_LIST_DATASET: k.bytes(16); k.string(); return true;
    case S(HBX_MSG_LIST_DATASET): {  // DatasetStateArray + ListH
      const uint32_t n = k.u32();
      if (k.ok) k.bytes(49ull * n);
      k.bytes(16);
      return true;
    }
    case HBX_MSG_ADD_DATASET_STATE: k.bytes(16); k.string(); k.bytes(48); return true;
    case HBX_MSG_REMOVE_DATASET_STATE: k.bytes(16); k.string(); k.bytes(16); return true;
    default:
      return false;
  }
}

// Parse the message at in[0..len).  Returns HBX_OK with m filled,
// HBX_ERR_CAPACITY if more bytes are needed (m->total_len is set once the
// block header is complete, else 0), HBX_ERR_FORMAT for an unknown type
// ("invalid protocol message received", protocol.go:253-256).
inline int parse(const uint8_t* in, uint64_t len, hbx_wire_msg* m) {
  std::memset(m, 0, sizeof(*m));
  hbxfmt::Reader r{in, len};
  const uint8_t* h = r.take(6);
  if (!h) return HBX_ERR_CAPACITY;
  m->num = (uint16_t)(h[0] << 8 | h[1]);
  m->type = (uint32_t)h[2] << 24 | (uint32_t)h[3] << 16 | (uint32_t)h[4] << 8 | h[5];
  const uint32_t t = m->type;
  if (is_block_msg(t)) {
    const uint8_t* id = r.take(16);
    const uint32_t nl = r.u32();
    if (!r.ok) return HBX_ERR_CAPACITY;
    m->n_links = nl;
    const uint64_t need = 6ull + 16 + 4 + 16ull * nl + 1 + 4;
    if (len < need) return HBX_ERR_CAPACITY;
    std::memcpy(m->id, id, 16);
    m->links = r.take(16ull * nl);
    m->data_type = r.u8();
    m->data_len = r.u32();
    m->header_len = need;
    m->total_len = need + m->data_len;
    if (len < m->total_len) return HBX_ERR_CAPACITY;
    m->data = in + need;
    return HBX_OK;
  }
  if (is_id_msg(t)) {
    m->header_len = m->total_len = 22;
    if (len < 22) return HBX_ERR_CAPACITY;
    std::memcpy(m->id, in + 6, 16);
    return HBX_OK;
  }
  Skip k{in + 6, len - 6};
  if (!walk_payload(t, k)) return HBX_ERR_FORMAT;
  if (!k.ok) return HBX_ERR_CAPACITY;
  m->header_len = 6;
  m->total_len = 6 + k.n;
  m->data = in + 6;
  m->data_len = (uint32_t)k.n;
  if (t == S(HBX_MSG_GREETING)) std::memcpy(m->id, in + 6, 16);
  if (t == S(HBX_MSG_ERROR)) {  // the text itself
    m->data = in + 10;
    m->data_len = (uint32_t)(k.n - 4);
    m->header_len = 10;
  }
  if (t == HBX_MSG_GREETING) {  // halo: the version
    m->data_len = (uint32_t)in[6] << 24 | (uint32_t)in[7] << 16 | (uint32_t)in[8] << 8 | in[9];
    m->header_len = 10;
    m->data = nullptr;
  }
  return HBX_OK;
}

}  // namespace hbxwire

// hbx_wire.h — the block-store subset of the Hashbox wire protocol (SURVEY
// §8f3), host side of libhbxgpu.  pkg/core/protocol.go:
//
//   ProtocolMessage  u16 Num | u32 Type | fields in declaration order
//                    (Serialize, protocol.go:184-203); client types are the
//                    lowercase constants, server replies the same & 0xDFDFDFDF
//                    (protocol.go:37-70)
//   allo / ACKN / read / READ   + BlockID (16)              (protocol.go:100-131)
//   writ / WRIT      + HashboxBlock.Serialize (block.go:56-69):
//                    BlockID | u32 #links | links | u8 DataType | u32 len | data
//   halo             + u32 Version;  HALO + SessionNonce (16);  quit: nothing
//   ERRS             + String (u32 len | bytes)
//
// Everything big-endian (pkg/core/utils.go:73-88).  The encoders write the
// fixed part only; a writ's data follows its header on the wire unchanged.
#pragma once

#include <cstdint>
#include <cstring>

#include "../../include/hbxgpu.h"
#include "hbx_formats.h"

namespace hbxwire {

constexpr uint32_t kServerMask = 0xDFDFDFDFu;  // protocol.go:67

inline bool is_id_msg(uint32_t t) {
  return t == HBX_MSG_ALLOCATE || t == HBX_MSG_READ || t == HBX_MSG_ACKNOWLEDGE ||
         t == (HBX_MSG_ALLOCATE & kServerMask) || t == (HBX_MSG_READ & kServerMask) ||
         t == (HBX_MSG_ACKNOWLEDGE & kServerMask);
}
inline bool is_block_msg(uint32_t t) { return t == HBX_MSG_WRITE || t == (HBX_MSG_WRITE & kServerMask); }

// Parse the message at in[0..len).  Returns HBX_OK with m filled,
// HBX_ERR_CAPACITY if more bytes are needed (m->total_len is set as soon as
// the header is complete, else 0), HBX_ERR_FORMAT for an unknown type
// ("invalid protocol message received", protocol.go:253-256).
inline int parse(const uint8_t* in, uint64_t len, hbx_wire_msg* m) {
  std::memset(m, 0, sizeof(*m));
  hbxfmt::Reader r{in, len};
  const uint8_t* h = r.take(6);
  if (!h) return HBX_ERR_CAPACITY;
  m->num = (uint16_t)(h[0] << 8 | h[1]);
  m->type = (uint32_t)h[2] << 24 | (uint32_t)h[3] << 16 | (uint32_t)h[4] << 8 | h[5];
  const uint32_t t = m->type;
  if (is_id_msg(t)) {
    m->header_len = 22;
  } else if (is_block_msg(t)) {
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
  } else if (t == HBX_MSG_GREETING) {
    m->header_len = 10;
  } else if (t == (HBX_MSG_GREETING & kServerMask)) {
    m->header_len = 22;
  } else if (t == HBX_MSG_GOODBYE || t == (HBX_MSG_GOODBYE & kServerMask)) {
    m->header_len = 6;
  } else if (t == (HBX_MSG_ERROR & kServerMask)) {
    const uint32_t sl = r.u32();
    if (!r.ok) return HBX_ERR_CAPACITY;
    m->header_len = 10;
    m->data_len = sl;
    m->total_len = 10ull + sl;
    if (len < m->total_len) return HBX_ERR_CAPACITY;
    m->data = in + 10;
    return HBX_OK;
  } else {
    return HBX_ERR_FORMAT;
  }
  m->total_len = m->header_len;
  if (len < m->total_len) return HBX_ERR_CAPACITY;
  if (is_id_msg(t) || t == (HBX_MSG_GREETING & kServerMask)) std::memcpy(m->id, in + 6, 16);
  if (t == HBX_MSG_GREETING) m->data_len = (uint32_t)in[6] << 24 | (uint32_t)in[7] << 16 | (uint32_t)in[8] << 8 | in[9];
  return HBX_OK;
}

}  // namespace hbxwire

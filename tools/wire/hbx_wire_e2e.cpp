// hbx_wire_e2e — the client's whole send path over a real socket (SURVEY
// §8f3): files on disk -> hbx_store_paths_z (rollsum split, block ids and a
// zlib stream per chunk on the GPU) -> the StoreBlock exchange of
// pkg/core/client.go:563-584 over loopback TCP to an in-process sink that
// answers like the server (server/server.go:160-202):
//
//   client  allo(id)          sink  READ(id)   if it does not hold the block
//                                   ACKN(id)   if it does (dedup)
//   client  writ(block)       sink  ACKN(id)   after re-verifying the block
//
// The sink re-verifies every k-th written block the way the server does
// (inflate, then HashData, block.go:152-174), with zlib and the CPU oracle's
// MD5 (oracle/hbx_oracle.c: the checker, not the thing measured).  Framing is
// the library's (hbx_wire_*).  Prints one JSON line.
//
// usage: hbx_wire_e2e <file-list> [io_threads] [window] [verify_every]
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>
#include <zlib.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hbxgpu.h"

extern "C" void hbxo_block_id(const uint8_t* links, uint32_t nlinks, const uint8_t* data, uint64_t len,
                              uint8_t out[16]);

namespace {

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool send_all(int fd, const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  while (n) {
    const ssize_t k = ::send(fd, b, n, MSG_NOSIGNAL);
    if (k <= 0) return false;
    b += k;
    n -= (size_t)k;
  }
  return true;
}

bool sendv_all(int fd, iovec* v, int cnt) {
  while (cnt) {
    ssize_t k = ::writev(fd, v, cnt);
    if (k <= 0) return false;
    while (cnt && (size_t)k >= v->iov_len) {
      k -= (ssize_t)v->iov_len;
      v++;
      cnt--;
    }
    if (cnt) {
      v->iov_base = static_cast<uint8_t*>(v->iov_base) + k;
      v->iov_len -= (size_t)k;
    }
  }
  return true;
}

// Buffered message reader over a socket.
struct Reader {
  int fd;
  std::vector<uint8_t> buf = std::vector<uint8_t>(1 << 20);
  size_t lo = 0, hi = 0;
  // next complete message (pointers valid until the next call); false on EOF/error
  bool next(hbx_wire_msg& m) {
    for (;;) {
      const int rc = hbx_wire_parse(buf.data() + lo, hi - lo, &m);
      if (rc == HBX_OK) {
        lo += m.total_len;
        return true;
      }
      if (rc != HBX_ERR_CAPACITY) return false;
      const size_t need = m.total_len ? m.total_len : 64;
      if (lo && (hi - lo) + need > buf.size() - lo) {  // compact
        std::memmove(buf.data(), buf.data() + lo, hi - lo);
        hi -= lo;
        lo = 0;
      }
      if (need > buf.size() - lo) buf.resize(lo + need + (1 << 20));
      const ssize_t k = ::recv(fd, buf.data() + hi, buf.size() - hi, 0);
      if (k <= 0) return false;
      hi += (size_t)k;
    }
  }
};

struct Block {
  const uint8_t* id;
  const uint8_t* z;  // zlib stream
  uint64_t zlen;
  uint64_t raw;  // uncompressed length
};

struct SinkStats {
  uint64_t allocs = 0, reads = 0, acks_dedup = 0, writes = 0, verified = 0, bad = 0, bytes = 0;
};

void sink(int fd, uint32_t verify_every, SinkStats* st) {
  Reader r{fd};
  std::set<std::string> have;
  std::vector<uint8_t> raw;
  hbx_wire_msg m;
  uint8_t out[22];
  while (r.next(m)) {
    if (m.type == HBX_MSG_GOODBYE) break;
    if (m.type == HBX_MSG_ALLOCATE) {
      st->allocs++;
      const bool known = have.count(std::string((const char*)m.id, 16)) != 0;
      const uint32_t t = (known ? HBX_MSG_ACKNOWLEDGE : HBX_MSG_READ) & HBX_SERVER_MASK;
      if (known) st->acks_dedup++; else st->reads++;
      hbx_wire_encode_id(m.num, t, m.id, out);
      if (!send_all(fd, out, 22)) break;
    } else if (m.type == HBX_MSG_WRITE) {
      st->writes++;
      st->bytes += m.data_len;
      if (verify_every && st->writes % verify_every == 1) {  // server.go:182 -> VerifyBlock
        raw.resize(8u << 20);
        uLongf n = raw.size();
        uint8_t id[16];
        const int zr = ::uncompress(raw.data(), &n, m.data, m.data_len);
        hbxo_block_id(m.links, m.n_links, raw.data(), n, id);
        st->verified++;
        if (zr != Z_OK || std::memcmp(id, m.id, 16) != 0) st->bad++;
      }
      have.insert(std::string((const char*)m.id, 16));
      hbx_wire_encode_id(m.num, HBX_MSG_ACKNOWLEDGE & HBX_SERVER_MASK, m.id, out);
      if (!send_all(fd, out, 22)) break;
    } else {
      break;
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <file-list> [io_threads] [window] [verify_every]\n", argv[0]);
    return 2;
  }
  const uint32_t io_threads = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 16u;
  const uint32_t window = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 4096u;
  const uint32_t verify_every = argc > 4 ? (uint32_t)std::atoi(argv[4]) : 64u;
  std::vector<std::string> names;
  {
    std::ifstream in(argv[1]);
    for (std::string line; std::getline(in, line);)
      if (!line.empty()) names.push_back(line);
  }
  const uint64_t n = names.size();
  std::vector<const char*> paths(n);
  std::vector<uint64_t> lens(n), caps(n), base(n), zbase(n);
  uint64_t ncap = 0, zcap = 0, total = 0;
  for (uint64_t i = 0; i < n; i++) {
    paths[i] = names[i].c_str();
    std::ifstream f(names[i], std::ios::binary | std::ios::ate);
    lens[i] = (uint64_t)f.tellg();
    total += lens[i];
    caps[i] = hbx_max_chunks(lens[i]);
    base[i] = ncap;
    ncap += caps[i];
    zbase[i] = zcap;
    zcap += hbx_deflate_file_bound(lens[i]);
  }
  std::vector<uint64_t> cuts(ncap), zoff(ncap), zlen(ncap);
  std::vector<uint8_t> ids(16 * ncap), zout(zcap + 16);
  std::vector<hbx_file_summary> sums(n);
  hbx_ctx* ctx = nullptr;
  if (hbx_ctx_create(0, &ctx) != HBX_OK) {
    std::fprintf(stderr, "hbx_ctx_create failed\n");
    return 1;
  }
  // warm-up on a few files (first-call costs: code objects, pinned staging)
  hbx_store_paths_z(ctx, std::min<uint64_t>(n, 64), paths.data(), lens.data(), cuts.data(), ids.data(),
                    base.data(), caps.data(), sums.data(), io_threads, 1ull << 30, zout.data(), zbase.data(),
                    zoff.data(), zlen.data());
  const double t0 = now();
  int rc = hbx_store_paths_z(ctx, n, paths.data(), lens.data(), cuts.data(), ids.data(), base.data(),
                             caps.data(), sums.data(), io_threads, 1ull << 30, zout.data(), zbase.data(),
                             zoff.data(), zlen.data());
  const double t1 = now();
  if (rc != HBX_OK) {
    std::fprintf(stderr, "hbx_store_paths_z: %s\n", hbx_last_error(ctx));
    return 1;
  }
  std::vector<Block> blocks;
  uint64_t zbytes = 0;
  for (uint64_t f = 0; f < n; f++) {
    uint64_t start = 0;
    for (uint32_t q = 0; q < sums[f].n_chunks; q++) {
      const uint64_t k = base[f] + q, e = cuts[k];
      blocks.push_back(Block{&ids[16 * k], zout.data() + zoff[k], zlen[k], e - start});
      zbytes += zlen[k];
      start = e;
    }
  }

  // loopback TCP: listener, sink thread, client (sender + receiver)
  const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  socklen_t al = sizeof(a);
  if (ls < 0 || ::bind(ls, (sockaddr*)&a, sizeof(a)) || ::listen(ls, 1) || ::getsockname(ls, (sockaddr*)&a, &al)) {
    std::perror("listen");
    return 1;
  }
  SinkStats st;
  std::thread srv([&] {
    const int fd = ::accept(ls, nullptr, nullptr);
    if (fd >= 0) {
      sink(fd, verify_every, &st);
      ::close(fd);
    }
  });
  const int cs = ::socket(AF_INET, SOCK_STREAM, 0);
  if (cs < 0 || ::connect(cs, (sockaddr*)&a, sizeof(a))) {
    std::perror("connect");
    return 1;
  }
  const int one = 1;
  ::setsockopt(cs, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));

  std::mutex mu;
  std::condition_variable cv;
  std::deque<uint32_t> to_write;  // blocks the server asked for (READ)
  uint64_t outstanding = 0, acked = 0, dedup = 0, written = 0;
  bool failed = false;
  const uint64_t nb = blocks.size();
  const double t2 = now();
  std::thread rx([&] {  // the client's receive side: READ -> queue the writ, ACKN -> done
    Reader r{cs};
    hbx_wire_msg m;
    while (r.next(m)) {
      std::lock_guard<std::mutex> g(mu);
      if (m.type == (HBX_MSG_READ & HBX_SERVER_MASK)) {
        to_write.push_back(m.num);  // the server wants this block's data
      } else if (m.type == (HBX_MSG_ACKNOWLEDGE & HBX_SERVER_MASK)) {
        acked++;
        outstanding--;
      } else {
        failed = true;
      }
      cv.notify_all();
      if (acked == nb) break;
    }
  });
  // sender: allo for every block (at most `window` unacknowledged), writ on demand
  uint64_t next = 0;
  std::vector<uint8_t> hdr(64);
  for (;;) {
    std::unique_lock<std::mutex> g(mu);
    cv.wait(g, [&] { return failed || !to_write.empty() || (next < nb && outstanding < window) || acked == nb; });
    if (failed || acked == nb) break;
    if (!to_write.empty()) {
      const uint32_t num = to_write.front();
      to_write.pop_front();
      g.unlock();
      // message numbers are block indices mod 2^16; with window < 65536 the
      // unacknowledged block with this number is unique
      uint64_t idx = (next - 1) - ((uint16_t)((uint16_t)(next - 1) - num));
      const Block& b = blocks[idx];
      uint64_t hn = 0;
      hbx_wire_encode_block_header((uint16_t)idx, HBX_MSG_WRITE, b.id, nullptr, 0, HBX_BLOCK_DATA_ZLIB,
                                   (uint32_t)b.zlen, hdr.data(), hdr.size(), &hn);
      iovec v[2] = {{hdr.data(), hn}, {const_cast<uint8_t*>(b.z), b.zlen}};
      if (!sendv_all(cs, v, 2)) break;
      written++;
    } else if (next < nb && outstanding < window) {
      outstanding++;
      const uint64_t idx = next++;
      g.unlock();
      uint8_t out[22];
      hbx_wire_encode_id((uint16_t)idx, HBX_MSG_ALLOCATE, blocks[idx].id, out);
      if (!send_all(cs, out, 22)) break;
    }
  }
  rx.join();
  const double t3 = now();
  uint8_t bye[6] = {0, 0, (uint8_t)(HBX_MSG_GOODBYE >> 24), (uint8_t)(HBX_MSG_GOODBYE >> 16),
                    (uint8_t)(HBX_MSG_GOODBYE >> 8), (uint8_t)HBX_MSG_GOODBYE};
  send_all(cs, bye, 6);
  srv.join();
  ::close(cs);
  ::close(ls);
  hbx_ctx_destroy(ctx);
  dedup = st.acks_dedup;
  std::printf(
      "{\"workload\": \"send path over loopback TCP: hbx_store_paths_z then allo/READ/writ/ACKN per chunk\", "
      "\"files\": %llu, \"bytes\": %llu, \"chunks\": %llu, \"compressed_bytes\": %llu, "
      "\"gpu_seconds\": %.3f, \"gpu_gibs\": %.3f, \"wire_seconds\": %.3f, \"wire_gbs_compressed\": %.3f, "
      "\"end_to_end_gibs\": %.3f, \"window\": %u, \"sink\": {\"allocs\": %llu, \"reads\": %llu, "
      "\"dedup_acks\": %llu, \"writes\": %llu, \"verified\": %llu, \"verify_failures\": %llu}, "
      "\"client_writes\": %llu, \"acked\": %llu, \"failed\": %s}\n",
      (unsigned long long)n, (unsigned long long)total, (unsigned long long)nb, (unsigned long long)zbytes,
      t1 - t0, total / (t1 - t0) / (1 << 30), t3 - t2, zbytes / (t3 - t2) / 1e9, total / (t3 - t0) / (1 << 30),
      window, (unsigned long long)st.allocs, (unsigned long long)st.reads, (unsigned long long)dedup,
      (unsigned long long)st.writes, (unsigned long long)st.verified, (unsigned long long)st.bad,
      (unsigned long long)written, (unsigned long long)acked, failed ? "true" : "false");
  return (failed || st.bad || acked != nb) ? 1 : 0;
}

// hbx_wire_e2e — the client's whole send path over a real socket (SURVEY
// §8d config 5, §8f3): files on disk -> hbx_store_paths_zcb (rollsum split,
// block ids and a zlib stream per chunk on the GPU; a callback per collected
// batch) -> the StoreBlock exchange of
// pkg/core/client.go:563-584 over loopback TCP to an in-process sink that
// answers like the server (server/server.go:160-202):
//
//   client  allo(id)          sink  READ(id)   if it does not hold the block
//                                   ACKN(id)   if it does (dedup)
//   client  writ(block)       sink  ACKN(id)   after re-verifying the block
//
// The sink re-verifies every written block before it acknowledges it, as the
// server does (server.go:180-182: VerifyBlock = inflate, then HashData,
// block.go:152-174), with zlib and the CPU oracle's MD5 (oracle/hbx_oracle.c:
// the checker, not the thing measured), on `verify_threads` verifier threads
// (the server verifies inline in the connection's goroutine; a pool keeps one
// core's inflate + MD5 rate from standing in for the GPU path's).  An ACKN is
// sent only once its block verified; a block that fails gets ERRS ("Unable to
// verify blockID", server.go:200-201).  verify_every > 1 samples every k-th
// write instead (a labelled second figure only).  Framing is the library's
// (hbx_wire_*).  Prints one JSON line.
//
// usage: hbx_wire_e2e <file-list> [io_threads] [window] [verify_every=1] [verify_threads=8]
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

// One written block waiting for its VerifyBlock (a copy: the reader's buffer
// moves on).
struct WriteJob {
  uint16_t num;
  uint8_t id[16];
  std::vector<uint8_t> links, data;
  uint32_t n_links;
  bool verify;
};

void sink(int fd, uint32_t verify_every, uint32_t verify_threads, SinkStats* st) {
  Reader r{fd};
  std::set<std::string> have;
  hbx_wire_msg m;
  uint8_t out[22];
  std::mutex send_mu, q_mu;
  std::condition_variable q_cv;
  std::deque<WriteJob> q;
  bool closing = false, dead = false;
  std::atomic<uint64_t> verified{0}, bad{0};
  auto reply = [&](uint16_t num, uint32_t type, const uint8_t* id) {
    uint8_t o[22];
    hbx_wire_encode_id(num, type & HBX_SERVER_MASK, id, o);
    std::lock_guard<std::mutex> g(send_mu);
    return send_all(fd, o, 22);
  };
  auto verifier = [&] {
    std::vector<uint8_t> raw(8u << 20);
    for (;;) {
      WriteJob j;
      {
        std::unique_lock<std::mutex> g(q_mu);
        q_cv.wait(g, [&] { return closing || !q.empty(); });
        if (q.empty()) return;
        j = std::move(q.front());
        q.pop_front();
      }
      q_cv.notify_all();  // room in the queue
      bool ok = true;
      if (j.verify) {  // server.go:182 -> VerifyBlock (block.go:152-166): inflate, HashData, compare
        uLongf n = raw.size();
        uint8_t id[16];
        const int zr = ::uncompress(raw.data(), &n, j.data.data(), j.data.size());
        hbxo_block_id(j.links.data(), j.n_links, raw.data(), n, id);
        ok = zr == Z_OK && std::memcmp(id, j.id, 16) == 0;
        verified++;
        if (!ok) bad++;
      }
      // ACKN after the verify; a failed one gets the server's error type
      if (!reply(j.num, ok ? HBX_MSG_ACKNOWLEDGE : HBX_MSG_ERROR, j.id)) {
        std::lock_guard<std::mutex> g(q_mu);
        dead = true;
      }
    }
  };
  std::vector<std::thread> pool;
  for (uint32_t t = 0; t < std::max(1u, verify_threads); t++) pool.emplace_back(verifier);
  while (r.next(m)) {
    if (m.type == HBX_MSG_GOODBYE) break;
    if (m.type == HBX_MSG_ALLOCATE) {
      st->allocs++;
      const bool known = have.count(std::string((const char*)m.id, 16)) != 0;
      if (known) st->acks_dedup++; else st->reads++;
      if (!reply(m.num, known ? HBX_MSG_ACKNOWLEDGE : HBX_MSG_READ, m.id)) break;
    } else if (m.type == HBX_MSG_WRITE) {
      st->writes++;
      st->bytes += m.data_len;
      WriteJob j;
      j.num = m.num;
      std::memcpy(j.id, m.id, 16);
      j.n_links = m.n_links;
      j.links.assign(m.links, m.links + 16u * m.n_links);
      j.data.assign(m.data, m.data + m.data_len);
      j.verify = verify_every != 0 && (st->writes - 1) % verify_every == 0;
      have.insert(std::string((const char*)m.id, 16));
      std::unique_lock<std::mutex> g(q_mu);
      q_cv.wait(g, [&] { return q.size() < 4u * pool.size() || dead; });  // bounded: the reader backs up
      if (dead) break;
      q.push_back(std::move(j));
      g.unlock();
      q_cv.notify_all();
    } else {
      break;
    }
  }
  {
    std::lock_guard<std::mutex> g(q_mu);
    closing = true;
  }
  q_cv.notify_all();
  for (auto& t : pool) t.join();
  st->verified = verified;
  st->bad = bad;
  (void)out;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <file-list> [io_threads] [window] [verify_every=1] [verify_threads=8]\n", argv[0]);
    return 2;
  }
  const uint32_t io_threads = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 16u;
  const uint32_t window = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 4096u;
  const uint32_t verify_every = argc > 4 ? (uint32_t)std::atoi(argv[4]) : 1u;  // server.go:182: every write
  const uint32_t verify_threads = argc > 5 ? (uint32_t)std::atoi(argv[5]) : 8u;
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
  // loopback TCP: listener, sink thread, client (sender + receiver); the
  // sender starts on a batch's blocks as soon as hbx_store_paths_zcb reports
  // the batch collected, so the wire overlaps the reading and hashing
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
      sink(fd, verify_every, verify_threads, &st);
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

  struct Shared {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<Block> blocks;       // grows as batches are collected (reserved: never moves)
    std::deque<uint32_t> to_write;   // message numbers the server asked for (READ)
    uint64_t outstanding = 0, acked = 0, written = 0, zbytes = 0;
    bool store_done = false, failed = false;
    const uint8_t* ids;
    const uint64_t* cuts;
    const uint64_t* base;
    const uint64_t* zoff;
    const uint64_t* zlen;
    const hbx_file_summary* sums;
    const uint8_t* zout;
  } S;
  S.blocks.reserve(ncap);
  S.ids = ids.data();
  S.cuts = cuts.data();
  S.base = base.data();
  S.zoff = zoff.data();
  S.zlen = zlen.data();
  S.sums = sums.data();
  S.zout = zout.data();
  auto ready = [](void* user, uint64_t first, uint64_t count) {
    Shared& S = *static_cast<Shared*>(user);
    std::lock_guard<std::mutex> g(S.mu);
    for (uint64_t f = first; f < first + count; f++) {
      uint64_t start = 0;
      for (uint32_t q = 0; q < S.sums[f].n_chunks; q++) {
        const uint64_t k = S.base[f] + q, e = S.cuts[k];
        S.blocks.push_back(Block{S.ids + 16 * k, S.zout + S.zoff[k], S.zlen[k], e - start});
        S.zbytes += S.zlen[k];
        start = e;
      }
    }
    S.cv.notify_all();
  };
  std::thread rx([&] {  // READ -> queue the writ; ACKN -> done
    Reader r{cs};
    hbx_wire_msg m;
    while (r.next(m)) {
      std::lock_guard<std::mutex> g(S.mu);
      if (m.type == (HBX_MSG_READ & HBX_SERVER_MASK)) {
        S.to_write.push_back(m.num);
      } else if (m.type == (HBX_MSG_ACKNOWLEDGE & HBX_SERVER_MASK)) {
        S.acked++;
        S.outstanding--;
      } else {
        S.failed = true;
      }
      S.cv.notify_all();
      if (S.store_done && S.acked == S.blocks.size()) break;
    }
  });
  std::thread tx([&] {  // allo for every block (at most `window` open), writ on demand
    uint64_t next = 0;
    std::vector<uint8_t> hdr(64);
    for (;;) {
      std::unique_lock<std::mutex> g(S.mu);
      S.cv.wait(g, [&] {
        return S.failed || !S.to_write.empty() || (next < S.blocks.size() && S.outstanding < window) ||
               (S.store_done && S.acked == S.blocks.size());
      });
      if (S.failed || (S.store_done && S.acked == S.blocks.size() && S.to_write.empty())) break;
      if (!S.to_write.empty()) {
        const uint32_t num = S.to_write.front();
        S.to_write.pop_front();
        // message numbers are block indices mod 2^16; fewer than 2^16 are open
        const uint64_t idx = (next - 1) - ((uint16_t)((uint16_t)(next - 1) - num));
        const Block b = S.blocks[idx];
        g.unlock();
        uint64_t hn = 0;
        hbx_wire_encode_block_header((uint16_t)idx, HBX_MSG_WRITE, b.id, nullptr, 0, HBX_BLOCK_DATA_ZLIB,
                                     (uint32_t)b.zlen, hdr.data(), hdr.size(), &hn);
        iovec v[2] = {{hdr.data(), hn}, {const_cast<uint8_t*>(b.z), b.zlen}};
        if (!sendv_all(cs, v, 2)) break;
        std::lock_guard<std::mutex> g2(S.mu);
        S.written++;
      } else if (next < S.blocks.size() && S.outstanding < window) {
        S.outstanding++;
        const uint64_t idx = next++;
        const uint8_t* id = S.blocks[idx].id;
        g.unlock();
        uint8_t out[22];
        hbx_wire_encode_id((uint16_t)idx, HBX_MSG_ALLOCATE, id, out);
        if (!send_all(cs, out, 22)) break;
      }
    }
  });
  const double t0 = now();
  int rc = hbx_store_paths_zcb(ctx, n, paths.data(), lens.data(), cuts.data(), ids.data(), base.data(),
                               caps.data(), sums.data(), io_threads, 1ull << 30, zout.data(), zbase.data(),
                               zoff.data(), zlen.data(), ready, &S);
  const double t1 = now();
  {
    std::lock_guard<std::mutex> g(S.mu);
    S.store_done = true;
    if (rc != HBX_OK) S.failed = true;
    S.cv.notify_all();
  }
  if (rc != HBX_OK) std::fprintf(stderr, "hbx_store_paths_zcb: %s\n", hbx_last_error(ctx));
  tx.join();
  const double t3 = now();
  // goodbye: the sink leaves its loop and closes, which ends the receiver
  uint8_t bye[6] = {0, 0, (uint8_t)(HBX_MSG_GOODBYE >> 24), (uint8_t)(HBX_MSG_GOODBYE >> 16),
                    (uint8_t)(HBX_MSG_GOODBYE >> 8), (uint8_t)HBX_MSG_GOODBYE};
  send_all(cs, bye, 6);
  if (S.failed) ::shutdown(cs, SHUT_RDWR);
  rx.join();
  const uint64_t nb = S.blocks.size(), zbytes = S.zbytes, acked = S.acked, written = S.written;
  const bool failed = S.failed;
  uint64_t dedup = 0;
  srv.join();
  ::close(cs);
  ::close(ls);
  hbx_ctx_destroy(ctx);
  dedup = st.acks_dedup;
  std::printf(
      "{\"workload\": \"send path over loopback TCP, overlapped: hbx_store_paths_zcb (per-batch callback) feeding "
      "allo/READ/writ/ACKN per chunk\", "
      "\"files\": %llu, \"bytes\": %llu, \"chunks\": %llu, \"compressed_bytes\": %llu, "
      "\"store_seconds\": %.3f, \"store_gibs\": %.3f, \"end_to_end_seconds\": %.3f, "
      "\"wire_tail_after_store_seconds\": %.3f, \"end_to_end_gibs\": %.3f, \"window\": %u, "
      "\"verify_every\": %u, \"verify_threads\": %u, "
      "\"sink\": {\"allocs\": %llu, \"reads\": %llu, \"dedup_acks\": %llu, \"writes\": %llu, "
      "\"verified\": %llu, \"verify_failures\": %llu}, \"client_writes\": %llu, \"acked\": %llu, "
      "\"failed\": %s}\n",
      (unsigned long long)n, (unsigned long long)total, (unsigned long long)nb, (unsigned long long)zbytes,
      t1 - t0, total / (t1 - t0) / (1 << 30), t3 - t0, t3 - t1, total / (t3 - t0) / (1 << 30), window,
      verify_every, verify_threads,
      (unsigned long long)st.allocs, (unsigned long long)st.reads, (unsigned long long)dedup,
      (unsigned long long)st.writes, (unsigned long long)st.verified, (unsigned long long)st.bad,
      (unsigned long long)written, (unsigned long long)acked, failed ? "true" : "false");
  return (failed || st.bad || acked != nb) ? 1 : 0;
}

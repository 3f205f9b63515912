// K7a + K7h (hbx_k7_deflate_size, hbx_k7_deflate_code) phase times on a Zipf-word text corpus: the
// kernel built with HBX_K7_PROBE=1 stamps (argv: MiB [random]) s_memtime at its phase boundaries
// (hbx_deflate.hip K7P); this prints the median cycles per phase over all
// segments, the kernel time and the coded size.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../hashbox_amd/csrc -o k7_phases k7_phases.hip
#define HBX_K7_PROBE 1
#include "hbx_deflate.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  const size_t total = (argc > 1 ? std::atol(argv[1]) : 256) << 20;  // MiB
  const size_t blk = 4u << 20;
  // corpus: words of 2-10 letters, Zipf(1.2) ranks over 5,000 words
  std::mt19937_64 rng(5);
  std::vector<std::string> vocab(5000);
  for (auto& w : vocab) {
    const int k = 2 + (int)(rng() % 9);
    for (int i = 0; i < k; i++) w.push_back((char)('a' + rng() % 26));
  }
  std::vector<double> cdf(vocab.size());
  double acc = 0;
  for (size_t i = 0; i < vocab.size(); i++) cdf[i] = (acc += 1.0 / std::pow((double)(i + 1), 1.2));
  std::uniform_real_distribution<double> u(0, acc);
  std::vector<uint8_t> text;
  text.reserve(total + 64);
  while (text.size() < total) {
    const auto& w = vocab[std::lower_bound(cdf.begin(), cdf.end(), u(rng)) - cdf.begin()];
    text.insert(text.end(), w.begin(), w.end());
    text.push_back(' ');
  }
  text.resize(total + 65536, 0);
  if (argc > 2 && std::string(argv[2]) == "random")
    for (auto& b : text) b = (uint8_t)(rng() >> 56);
  uint8_t* d_in;
  (void)hipMalloc(&d_in, text.size());
  (void)hipMemcpy(d_in, text.data(), text.size(), hipMemcpyHostToDevice);
  std::vector<hbxz::ZBlock> zb;
  uint32_t nseg = 0;
  for (size_t o = 0; o < total; o += blk) {
    const uint64_t len = std::min(blk, total - o);
    const uint32_t ns = (uint32_t)((len + hbxz::kSeg - 1) / hbxz::kSeg);
    zb.push_back(hbxz::ZBlock{reinterpret_cast<uint64_t>(d_in + o), 0, len, nseg, ns});
    nseg += ns;
  }
  hbxz::ZBlock* d_zb;
  hbxz::SegInfo* d_info;
  uint32_t* d_img;
  (void)hipMalloc(&d_zb, zb.size() * sizeof(hbxz::ZBlock));
  (void)hipMalloc(&d_info, nseg * sizeof(hbxz::SegInfo));
  (void)hipMalloc(&d_img, (size_t)nseg * hbxz::kSlot);
  (void)hipMemcpy(d_zb, zb.data(), zb.size() * sizeof(hbxz::ZBlock), hipMemcpyHostToDevice);
  // K7e first (as the engine does): it stores incompressible segments, K7a parses the rest
  hipLaunchKernelGGL(hbx_k7_deflate_entropy, dim3(nseg), dim3(hbxz::kEThreads), 0, 0, d_zb, (uint32_t)zb.size(), nseg,
                     d_info);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 3; rep++) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(hbx_k7_deflate_size, dim3(nseg), dim3(hbxz::kThreads), 0, 0, d_zb, (uint32_t)zb.size(), nseg,
                       d_info, d_img);
    hipLaunchKernelGGL(hbx_k7_deflate_code, dim3(nseg), dim3(hbxz::kThreads), 0, 0, d_zb, (uint32_t)zb.size(), nseg,
                       d_info, d_img);
    (void)hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) {
      std::fprintf(stderr, "launch failed\n");
      return 1;
    }
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  std::vector<hbxz::SegInfo> info(nseg);
  (void)hipMemcpy(info.data(), d_info, nseg * sizeof(hbxz::SegInfo), hipMemcpyDeviceToHost);
  const uint32_t np = std::min<uint32_t>(nseg, 1u << 16);
  std::vector<unsigned long long> pr((size_t)np * 16);
  (void)hipMemcpyFromSymbol(pr.data(), HIP_SYMBOL(hbx_k7_probe), pr.size() * 8);
  uint64_t out = 0;
  uint32_t modes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (auto& x : info) {
    out += x.bytes;
    modes[x.mode & 7u]++;
  }
  std::printf("# %u segments, %.1f MiB text, K7a+K7h %.3f ms = %.2f GB/s, coded/input %.4f, modes stored/fixed/dyn/src-stored/group-head/group-member %u/%u/%u/%u/%u/%u\n",
              nseg, total / 1048576.0, ms, total / (ms * 1e6), (double)out / total, modes[0], modes[1], modes[2], modes[3],
              modes[4], modes[5]);
  // K7a: 0..5; K7h: 6 (start) .. 7 (emission) .. 15 (end)
  const int ph2[][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4}, {4, 5}, {6, 7}, {7, 15}};
  const char* names[] = {"load+init", "history inserts", "candidates", "dry parse+handoff", "final parse",
                         "K7h reload+code", "K7h emit+copy"};
  for (int ph = 0; ph < 7; ph++) {
    std::vector<double> v;
    const int a = ph2[ph][0], b = ph2[ph][1];
    for (uint32_t g = 0; g < np; g++)
      if (pr[16 * g + b] >= pr[16 * g + a] && pr[16 * g + a] != 0) v.push_back((double)(pr[16 * g + b] - pr[16 * g + a]));
    std::sort(v.begin(), v.end());
    if (v.empty()) continue;
    std::printf("%-20s median %10.0f  p90 %10.0f cycles (n=%zu)\n", names[ph], v[v.size() / 2], v[v.size() * 9 / 10], v.size());
  }
  // inside K7h's code build (dynamic code only; a group's pass, or the segment's own): 14 -> 8 sort,
  // 8 -> 9 trees, 9 -> 10 lengths and codes, 10 -> 11 header runs, 11 -> 7 costs and the group decision
  const int sub[][2] = {{14, 8}, {8, 9}, {9, 10}, {10, 11}, {11, 7}, {6, 12}, {12, 13}, {13, 14}, {14, 8}};
  const char* sn[] = {"  huff: sort", "  huff: trees", "  huff: lengths", "  huff: header rle", "  huff: costs",
                      "    sort: sums", "    sort: entropy", "    sort: init", "    sort: rank"};
  for (int i = 0; i < 9; i++) {
    std::vector<double> v;
    for (uint32_t g = 0; g < np; g++) {
      const unsigned long long a = pr[16 * g + sub[i][0]], b = pr[16 * g + sub[i][1]];
      if (a && b >= a) v.push_back((double)(b - a));
    }
    std::sort(v.begin(), v.end());
    if (!v.empty()) std::printf("%-20s median %10.0f cycles (n=%zu)\n", sn[i], v[v.size() / 2], v.size());
  }
  return 0;
}

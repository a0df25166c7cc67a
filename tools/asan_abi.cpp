// Host-side sanitizer run of the C ABI: linked against
// libaccunet_hip_asan.so, whose entry-point sources are compiled with
// -Xarch_host -fsanitize=address (acc-unet-unext_amd/Makefile, target `asan`).
// Exercises every entry point that answers on the host without touching a device:
// geometry / workspace-size queries over a sweep of shapes (incl. the BASELINE configs
// and ragged edges), the per-stream ticket-bank table (fill it, overflow it, unregister
// in every position), the ABI hash, and the argument checks that return -2 before any
// launch. AddressSanitizer aborts the process on any out-of-bounds or use-after-free
// access in that host code; the exit code is 0 only if every call also returned what
// include/accunet.h promises.
//   make -C acc-unet-unext_amd asan && tools/asan_abi   (tests/test_host_cpu.py)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/accunet.h"

static int fails = 0;
#define EXPECT(c)                                               \
  do {                                                          \
    if (!(c)) {                                                 \
      std::fprintf(stderr, "%s:%d EXPECT(%s)\n", __FILE__, __LINE__, #c); \
      ++fails;                                                  \
    }                                                           \
  } while (0)

int main() {
  // shapes: (B, H, W, C) of every HANC width at the BASELINE configs plus ragged ones
  const int shapes[][4] = {{16, 256, 256, 96}, {16, 256, 256, 9},  {16, 128, 128, 192},
                           {16, 64, 64, 384},  {16, 64, 64, 4352}, {16, 32, 32, 768},
                           {16, 16, 16, 1536}, {4, 512, 512, 96},  {1, 128, 128, 96},
                           {2, 13, 35, 96},    {1, 8, 17, 256},    {2, 6, 300, 8},
                           {3, 5, 5, 32},      {1, 1, 1, 4}};
  long sink = 0;
  for (auto& s : shapes) {
    for (int dt = 0; dt < 2; ++dt) {
      const int r = accunet_dw3x3_rows(s[0], s[1], s[2], s[3], dt, dt);
      EXPECT(r > 0);
      sink += r;
      sink += (long)accunet_dw3x3_wgrad_ws(s[0], s[1], s[2], s[3], dt);
    }
    for (int dt = 0; dt < 2; ++dt) {
      const int v = accunet_dw3x3_variant(s[0], s[1], s[2], s[3], dt);
      EXPECT(v >= 0 && v <= 4);  // 4: the 16-row one-shot tiles
    }
    const long P = (long)s[0] * s[1] * s[2];
    sink += accunet_stream_rows(P, s[3]);
    sink += (long)accunet_bn_bwd_ws_elems(P, s[3]);
    sink += (long)accunet_bn_bwd_part_ws_elems(P, 64, s[3]);
    sink += (long)accunet_head_ws_elems(P, s[3]);
    sink += accunet_se_stats_rows(s[0], s[1] * s[2], s[3]);
    sink += (long)accunet_se_ws_elems(s[0], s[1] * s[2], s[3], s[3] / 8 ? s[3] / 8 : 1);
    sink += (long)accunet_se_save_elems(s[0], s[3], s[3] / 8 ? s[3] / 8 : 1);
    sink += accunet_layernorm_rows(P);
    for (int am = 0; am < 3; ++am)
      for (int bm = 0; bm < 3; ++bm) sink += accunet_gemm_stats_rows((int)P, s[3], 64, am, bm, 32);
  }
  for (int b = 1; b <= 32; b *= 2) sink += (long)accunet_loss_ws_elems(b);
  EXPECT(accunet_adam_chunk_elems() > 0);
  EXPECT(accunet_relayout_blocks(1) == 1 && accunet_relayout_blocks(1024) == 1 &&
         accunet_relayout_blocks(1025) == 2);
  EXPECT(accunet_relayout_batch(nullptr, 4, 4, nullptr) == -2);
  // dwconv2d geometry: every odd k of the reference's test.py, both paddings
  for (int k = 3; k <= 31; k += 2)
    for (int rep = 0; rep < 2; ++rep) {
      int oh = -1, ow = -1;
      EXPECT(accunet_dwconvk_out_hw(64, 64, k, k, k / 2, k / 2, &oh, &ow) == 0);
      EXPECT(oh == 64 && ow == 64);
      sink += (long)accunet_dwconvk_dgrad_ws(64, 384, 64, 64, k, k, k / 2, k / 2, rep);
      sink += (long)accunet_dwconvk_wgrad_ws(64, 384, 64, 64, k, k, k / 2, k / 2);
    }
  {
    int oh, ow;
    EXPECT(accunet_dwconvk_out_hw(8, 8, 33, 3, 1, 1, &oh, &ow) != 0);  // kh > 31
  }
  // ticket-bank table: 64 fake handles (table keys only, never dereferenced), one too
  // many, re-registration, unregister from the middle / ends, and reuse of freed slots
  std::vector<void*> hs;
  for (int i = 0; i < 65; ++i) hs.push_back(reinterpret_cast<void*>(0x1000 + 16 * i));
  for (int i = 0; i < 64; ++i) EXPECT(accunet_stream_ticket_bank(hs[i], i & 1) == 0);
  EXPECT(accunet_stream_ticket_bank(hs[64], 1) == -2);  // table full
  EXPECT(accunet_stream_ticket_bank(hs[10], 0) == 0);   // re-registration overwrites
  EXPECT(accunet_stream_ticket_unregister(hs[0]) == 0);
  EXPECT(accunet_stream_ticket_unregister(hs[63]) == 0);
  EXPECT(accunet_stream_ticket_unregister(hs[31]) == 0);
  EXPECT(accunet_stream_ticket_unregister(hs[31]) == -2);
  EXPECT(accunet_stream_ticket_bank(hs[64], 1) == 0);  // a freed slot is reused
  for (int i = 0; i < 65; ++i) accunet_stream_ticket_unregister(hs[i]);
  EXPECT(accunet_stream_ticket_unregister(hs[5]) == -2);
  EXPECT(accunet_stream_ticket_bank(nullptr, 1) == -2);
  EXPECT(accunet_stream_ticket_bank(hs[1], 2) == -2);
  EXPECT(accunet_stream_ticket_unregister(nullptr) == -2);
  // argument checks that answer before any launch
  EXPECT(accunet_gemm(nullptr, nullptr, 0, nullptr) == -2);
  float* one = reinterpret_cast<float*>(16);
  EXPECT(accunet_dw3x3_fwd(one, one, nullptr, nullptr, nullptr, 0, 1, one, nullptr, 1, 8, 8, 32,
                           one, nullptr, 0, 0, nullptr) == -2);
  EXPECT(accunet_abi_hash() != 0);
  std::printf("asan_abi: %d failure(s), checksum %ld\n", fails, sink);
  return fails ? 1 : 0;
}

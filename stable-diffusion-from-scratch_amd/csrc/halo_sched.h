// Host-side plan of the halo-tile 3x3 conv (conv.hip conv_halo_kernel, variants 36 / 37).
//
// A 3x3 pad-0 conv over a zero-bordered NHWC image ([B, ho+2, wo+2, C], written by
// sdk_group_norm_apply_padded) runs as an implicit GEMM whose K-step is (64-channel block cb,
// tap ky*3+kx).  The LDS-DMA kernels gather the shifted pixel window of every tap: nine A-tile
// DMAs per channel block.  The halo kernel instead stages, per channel block, the padded input
// rows its M-tile touches (one contiguous span of whole padded rows) ONCE, as 1-KiB pieces
// (8 pixels x 64 channels) in an LDS ring, and forms all nine taps' A fragments from it with
// per-tap offsets (h = row * hs + col + ky * hs + kx in halo pixels).
//
// The ring is cut in pieces, not rows: pieces of block cb+1 are streamed in while block cb still
// reads its own, each into the slot of a piece that is already dead.  Piece q of a block holds
// halo pixels [8q, 8q+8); it is first read by the smallest tap row ky that reads any of its rows
// (`need`, the K-step 3*ky) and last read by the largest (`dead`, K-step 3*ky+2).  Global piece
// g = cb*np + q lives in slot g % rp, i.e. piece q of cb+1 replaces piece q - (rp - np) of cb.
// The issue schedule tau(q) (K-step relative to the piece's own block start, negative = during
// the previous block) is greedy-earliest subject to: the slot's previous occupant is dead,
// tau is monotone in q, at most `cap` pieces per K-step (a block's tau and its successor's tau - 9
// are the same K-step), and tau(q) <= need(q) - lead (the K-step that reads a piece waits for DMAs
// issued at least one K-step before it; the GroupNorm-fused form needs one more for the transform).  The kernel issues,
// at K-step j of block cb, the global pieces [cb*np + phi[j], cb*np + phi[j+1]).
//
// Header-only, no HIP: tests/test_halo_schedule.py compiles it with g++ and replays the ring.
#pragma once

#include <algorithm>
#include <vector>

namespace sdk {

struct HaloPlan {
  int hs = 0;        // halo row stride in pixels (= the padded source width wo + 2)
  int rh = 0;        // halo rows per tile (worst case over the tiles)
  int np = 0;        // 1-KiB pieces per channel block
  int rp = 0;        // ring slots (pieces)
  int phi[10] = {};  // pieces issued before K-step j of a block, relative to cb*np (phi[9] = np + phi[0])
};

// Rows of output pixels a tile of `tbm` consecutive pixels spans, and the halo geometry.
// src_h / src_w: the padded source (ho + 2, wo + 2).  Returns 0 when the plan exists.
//   multi-image tiles: tbm % hw == 0 (whole images per tile); single-image: hw % tbm == 0.
// lead: K-steps between a piece's issue and its first read (1: read as landed; 2: the GroupNorm-fused
// form transforms a piece in LDS the K-step after it lands, before it is read)
inline int halo_plan(int hw, int ho, int wo, int src_h, int src_w, int tbm, int max_rp, int cap, HaloPlan* out,
                     int lead = 1) {
  if (src_h != ho + 2 || src_w != wo + 2 || hw != ho * wo || tbm <= 0 || cap <= 0) return 1;
  const bool multi = tbm % hw == 0;
  if (!multi && hw % tbm) return 2;
  int R = 0, rh = 0;
  if (multi) {
    R = ho;
    rh = (tbm / hw) * src_h;
  } else {
    for (int k = 0; k < hw / tbm; ++k) {        // every tile start column inside an image
      const int c0 = (k * tbm) % wo;
      R = std::max(R, (c0 + tbm + wo - 1) / wo);
    }
    rh = R + 2;
  }
  const int hs = src_w;
  const long long L = (long long)rh * hs;
  const int np = (int)((L + 7) / 8);
  if (np > max_rp) return 3;
  // taps (ky) that read halo row hr: the rows of output-row index lr = hr - ky present in a tile
  auto ky_range = [&](int hr, int& lo, int& hi) {
    const int hl = multi ? hr % src_h : hr;   // row inside its image's padded rows
    lo = std::max(0, hl - R + 1);
    hi = std::min(2, hl);
  };
  std::vector<int> need(np), dead(np);
  for (int q = 0; q < np; ++q) {
    const int r0 = (8 * q) / hs, r1 = std::min(rh - 1, (8 * q + 7) / hs);
    int nd = 1 << 20, dd = -1;
    for (int hr = r0; hr <= r1; ++hr) {
      int lo, hi;
      ky_range(hr, lo, hi);
      if (lo > hi) continue;                      // a padding row no tap of this tile reads
      nd = std::min(nd, 3 * lo);
      dd = std::max(dd, 3 * hi + 2);
    }
    if (dd < 0) { nd = 8; dd = -1; }              // never read: any time, dead at once
    need[q] = nd;
    dead[q] = dd;
  }
  // the largest ring that fits gives the most lead time
  const int rp = max_rp;
  const int ep = rp - np;
  std::vector<int> tau(np);
  int cnt[9] = {};                                // pieces per K-step of a block (tau and tau - 9 coincide)
  int prev = -9;
  for (int q = 0; q < np; ++q) {
    int lo = q >= ep ? dead[q - ep] - 8 : -9;     // the occupant (cb-1, q-ep) died at K-step dead - 9
    lo = std::max(std::max(lo, prev), -9);
    while (lo <= 8 && cnt[(lo + 9) % 9] >= cap) ++lo;
    if (lo > 8 || lo > need[q] - lead) return 4;  // not in time: the ring is too small for this tile
    tau[q] = lo;
    ++cnt[(lo + 9) % 9];
    prev = lo;
  }
  out->hs = hs;
  out->rh = rh;
  out->np = np;
  out->rp = rp;
  for (int j = 0; j <= 9; ++j) {
    int c = 0;
    for (int q = 0; q < np; ++q) c += (tau[q] < j) + (tau[q] < j - 9);
    out->phi[j] = c;
  }
  return 0;
}

}  // namespace sdk

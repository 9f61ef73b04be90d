// CPU replay of the halo-tile conv's LDS ring (conv.hip conv_halo_kernel, plan from halo_sched.h):
// the per-wave issue state machine of the kernel, then every A-fragment read of every K-step of every
// tile is checked to find (a) its own block's piece in the slot, (b) a piece issued at least one K-step
// earlier (the counted vmcnt wait covers only those), (c) the padded input pixel the tap addresses.
// usage: halo_sim batch ho wo tbm nw max_rp ncb split [lead]  -> prints "OK np rp phi..." or "FAIL ..."
// lead 2 (the GroupNorm-fused form): a piece is also transformed in LDS at the K-step after its issue, so
// it must be issued at least two K-steps before its first read.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "halo_sched.h"

using namespace sdk;

int main(int argc, char** argv) {
  if (argc != 9 && argc != 10) return 2;
  const int lead = argc == 10 ? atoi(argv[9]) : 1;
  const int batch = atoi(argv[1]), ho = atoi(argv[2]), wo = atoi(argv[3]), tbm = atoi(argv[4]);
  const int nw = atoi(argv[5]), max_rp = atoi(argv[6]), ncb = atoi(argv[7]), split_req = atoi(argv[8]);
  const int hw = ho * wo, M = batch * hw, sh = ho + 2, sw_ = wo + 2;
  HaloPlan hp;
  const int rc = halo_plan(hw, ho, wo, sh, sw_, tbm, max_rp, nw, &hp, lead);
  if (rc) {
    printf("NOPLAN %d\n", rc);
    return 0;
  }
  const int NP = hp.np, RP = hp.rp, HS = hp.hs;
  const int kt_total = 9 * ncb;
  const int split = split_req < 1 ? 1 : (split_req > ncb ? ncb : split_req);
  const int kt_per_split = 9 * ((ncb + split - 1) / split);
  const int tiles_m = (M + tbm - 1) / tbm;
  long long reads = 0;
  for (int tm = 0; tm < tiles_m; ++tm) {
    const int m0 = tm * tbm;
    const int b0 = m0 / hw, oy0 = (m0 - b0 * hw) / wo, hstart = (b0 * sh + oy0) * sw_;
    for (int kt0 = 0; kt0 < kt_total; kt0 += kt_per_split) {
      const int kt1 = kt0 + kt_per_split < kt_total ? kt0 + kt_per_split : kt_total;
      const int cb0 = kt0 / 9, gend = ((kt1 + 8) / 9) * NP;
      std::vector<long long> ring(RP, -1);
      std::vector<int> issued_at((size_t)(ncb + 2) * NP, 1 << 30);
      struct W { int gw, cbw, qw, sw; };
      std::vector<W> wav(nw);
      for (int w = 0; w < nw; ++w) wav[w] = {cb0 * NP + w, cb0, w, (cb0 * NP + w) % RP};
      auto issue = [&](int hi, int when) {
        for (int w = 0; w < nw; ++w) {
          W& s = wav[w];
          while (s.gw < hi) {
            if (s.cbw * NP + s.qw != s.gw || s.sw != s.gw % RP || s.qw < 0 || s.qw >= NP) {
              printf("FAIL wave state g=%d cb=%d q=%d slot=%d\n", s.gw, s.cbw, s.qw, s.sw);
              exit(1);
            }
            ring[s.sw] = s.gw;
            issued_at[s.gw] = when;
            s.gw += nw;
            s.qw += nw;
            if (s.qw >= NP) { s.qw -= NP; ++s.cbw; }
            s.sw += nw;
            if (s.sw >= RP) s.sw -= RP;
          }
        }
      };
      issue(std::min(gend, cb0 * NP + hp.phi[0]), kt0 - 10);   // prologue: waited (and transformed) before the loop
      int cb = cb0, j = 0, cbslot = (cb0 * NP) % RP;
      for (int kt = kt0; kt < kt1; ++kt) {
        issue(std::min(gend, cb * NP + hp.phi[j + 1]), kt);
        const int ky = j / 3, kx = j - 3 * ky, toff = ky * HS + kx;
        for (int pix = 0; pix < tbm; ++pix) {
          const int m = m0 + pix < M ? m0 + pix : M - 1;
          const int b = m / hw, rem = m - b * hw, oy = rem / wo, ox = rem - oy * wo;
          const int h = ((b - b0) * sh + oy - oy0) * HS + ox + toff;
          if (h < 0 || h >= hp.rh * HS) { printf("FAIL halo index %d outside %d rows\n", h, hp.rh); return 1; }
          if (hstart + h != (b * sh + oy + ky) * sw_ + ox + kx) { printf("FAIL pixel map\n"); return 1; }
          int slot = cbslot + (h >> 3);
          if (slot >= RP) slot -= RP;
          const long long want = (long long)cb * NP + (h >> 3);
          if (ring[slot] != want) {
            printf("FAIL tile %d kt %d pix %d: slot %d holds %lld, want %lld\n", tm, kt, pix, slot, ring[slot], want);
            return 1;
          }
          if (issued_at[want] > kt - lead) {
            printf("FAIL tile %d kt %d: piece %lld issued at %d (not before the read)\n", tm, kt, want,
                   issued_at[want]);
            return 1;
          }
          ++reads;
        }
        if (++j == 9) {
          j = 0;
          ++cb;
          cbslot += NP;
          if (cbslot >= RP) cbslot -= RP;
        }
      }
    }
  }
  printf("OK np=%d rp=%d rh=%d reads=%lld phi=", NP, RP, hp.rh, reads);
  for (int j = 0; j <= 9; ++j) printf("%d%c", hp.phi[j], j < 9 ? ',' : '\n');
  return 0;
}

// Host check of the SYRK t-slice table (syrk_t_table): for nb = 1..12 every K column is
// covered exactly once, by a group that holds its panel.  build: hipcc -std=c++17 -o
// syrk_tmap_check syrk_tmap_check.hip ; run on any host (no kernel is launched).
#include "../../sparsergps_amd/csrc/k_mfma.hip"
#include <cstdio>
int main() {
  int bad = 0;
  for (int nb = 1; nb <= 12; ++nb) {
    const int T = nb * (nb - 1) / 2 + (3 * nb + 3) / 4;
    int tmap[128];
    const int S = syrk_t_table(nb, T, tmap);
    if (S == 0) { printf("nb %d: no table\n", nb); ++bad; continue; }
    const int W = 128 / S;
    std::vector<int> cover(nb * 128, 0);
    for (int gi = 0; gi < T; ++gi) {
      if (tmap[gi] < 0) continue;
      const int p = tmap[gi] / S, sl = tmap[gi] % S;
      int ta, tb; syrk_group_panels(gi, nb, ta, tb);
      if (p != ta && p != tb) { printf("nb %d gi %d: panel %d not held\n", nb, gi, p); ++bad; }
      for (int c = 0; c < W; ++c) cover[p * 128 + sl * W + c]++;
    }
    for (int i = 0; i < nb * 128; ++i) if (cover[i] != 1) { printf("nb %d col %d covered %d\n", nb, i, cover[i]); ++bad; break; }
    printf("nb %2d groups %2d S %d\n", nb, T, S);
  }
  return bad;
}

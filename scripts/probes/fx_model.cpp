// Host-only model of the factorised planner (fx_build, fx_skew): reads a
// [D][C] int32 delay table (raw file) and prints the plan's pattern count,
// modelled costs, staged elements and chunk counts with and without the
// delay-aligned tiles.  Developer tool (no GPU): build with
//   hipcc --cuda-host-only -O2 -std=c++17 -x hip scripts/probes/fx_model.cpp -o build/fx_model
#include "../../pypulsar_amd/csrc/pdd_sweep.hip"
#include <cstdio>

int main(int argc, char** argv) {
  if (argc < 4) { fprintf(stderr, "usage: fx_model table.bin D C [g]\n"); return 2; }
  const int64_t D = atoll(argv[2]), C = atoll(argv[3]);
  const int g = argc > 4 ? atoi(argv[4]) : 4;
  std::vector<int32_t> tab((size_t)(D * C));
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(tab.data(), 4, tab.size(), f) != tab.size()) { fprintf(stderr, "bad table\n"); return 2; }
  fclose(f);
  const Variant v = kU8FxVariants[0];
  const int64_t room = lds_budget(v) - il_meta_bytes(v.NBUF, v.CC, v.DB());
  const int64_t buf = std::max<int64_t>(0, room / (v.NBUF * 16) / 64 * 64);
  for (int skew = 0; skew < 2; ++skew)
    for (int pairs = 1; pairs >= 0; --pairs) {
      FxTables T;
      const bool ok = fx_build(tab.data(), D, C, v, buf, g, true, T, pairs, skew);
      int64_t nch = 0, nwin = 0, el = 0;
      const int64_t nb = cdiv(D, v.DB());
      for (int64_t b = 0; b < nb; ++b) nch += ok ? T.cht[(size_t)(b * (T.maxch + 1))] : 0;
      for (int64_t b = 0; ok && b < nb; ++b)
        for (int k = 0; k < T.cht[(size_t)(b * (T.maxch + 1))]; ++k)
          for (int i = 0; i < kFxWin; ++i) {
            const int* r = &T.wt[(((size_t)b * T.maxch + k) * kFxWin + i) * 4];
            if (r[1] == 0 || (r[3] & 0xfffff) == T.n_pat) continue;  // empty / pad group
            ++nwin;
            el += r[1];
          }
      if (ok)
        printf("  windows per (block, group) %.2f, mean window %.1f elements (Tq %d + span %.1f)\n",
               (double)nwin / (nb * (C / g)), (double)el / nwin, 64 * v.G, (double)el / nwin - 64 * v.G);
      printf("skew %d pairs %d ok %d: n_pat %lld cost_f %.4g cost_b %.4g el_f/tile %.4g chunks/blk %.1f "
             "pair_ratio %.5f sig_max %d lo %d hi %d\n",
             skew, pairs, (int)ok, (long long)T.n_pat, T.cost_f, T.cost_b, T.el_f, (double)nch / nb,
             T.pair_ratio, T.sig_max, T.lo_f, T.hi_f);
    }
  return 0;
}

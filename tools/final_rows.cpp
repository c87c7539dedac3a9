// Host tool: final-pass (S/N) units of a config's schedule -- output rows per
// unit and whether they fit the wide S/N stride (ffa_kernels.hip
// snr_wide_stride) for a widest boxcar wmax.
// hipcc -O2 -I riptide_amd/csrc tools/final_rows.cpp riptide_amd/csrc/plan.cpp -o /tmp/final_rows
// /tmp/final_rows N TSAMP PMIN PMAX BMIN BMAX WMAX
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#include "plan.hpp"

using namespace rt;

int main(int argc, char** argv)
{
    PgramParams a;
    a.size = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1u << 22);
    a.tsamp = argc > 2 ? std::atof(argv[2]) : 256e-6;
    a.pmin = argc > 3 ? std::atof(argv[3]) : 0.2;
    a.pmax = argc > 4 ? std::atof(argv[4]) : 5.0;
    a.bmin = argc > 5 ? std::atoi(argv[5]) : 240;
    a.bmax = argc > 6 ? std::atoi(argv[6]) : 260;
    const int wmax = argc > 7 ? std::atoi(argv[7]) : 42;
    PgramPlan pg;
    build_pgram_plan(a, pg);
    std::vector<FfaXform> xf;
    for (const Step& s : pg.steps) {
        if (!s.rows_eval) continue;
        FfaXform X{};
        X.p = s.bins;
        X.m = s.rows;
        X.rows_eval = s.rows_eval;
        X.snr_row = s.out_row;
        xf.push_back(X);
    }
    ExecPlan ex;
    build_exec_plan(xf, true, 10, 1ull << 40, ex, std::getenv("NOCAP") ? 0u : (uint32_t)wmax);
    double rows = 0, rows_fit = 0, rows_whole = 0, rows_noblob = 0, units = 0;
    std::map<int, double> hist;
    for (const ConeItem& it : ex.items) {
        if (it.dst != kSelSnr) continue;
        const int p = (int)ex.xf[it.xform].p;
        const int n0 = it.mode == kModeTile ? (int)(it.s1 - it.s0) : (int)it.node_size;
        const double r = n0;
        units += 1;
        rows += r;
        if (it.levels == 0 || it.pad == kNoBlob) { rows_noblob += r; continue; }
        if (it.mode == kModeWhole) rows_whole += r;
        if ((double)n0 * snr_wide_stride(p, wmax) <= kLdsDataFloats) rows_fit += r;
        hist[n0 / 8 * 8] += r;
    }
    std::printf("final units %.0f rows %.0f: fit wide stride %.1f%%, whole-unit rows %.1f%%, no slots/levels %.1f%%\n",
                units, rows, 100 * rows_fit / rows, 100 * rows_whole / rows, 100 * rows_noblob / rows);
    for (auto& kv : hist) std::printf("  n0 %3d-%3d: %5.1f%% of rows\n", kv.first, kv.first + 7, 100 * kv.second / rows);
}

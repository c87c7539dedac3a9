// Host-only wave balance of the 4/5-slot row-slot steps of a periodogram's
// cone schedule: per merge step, every wave's slots (slot g on wave g mod 8)
// weighted by the LDS reads their kind costs in a two-level step (one row 4,
// a pair 5 -- its second row by DPP --, a half 6, two rows 8); reports the
// step's critical path (the busiest wave) against the mean, summed over the
// units of every 4/5-slot launch.  Build (host only):
//   g++ -O2 -std=c++17 -I riptide_amd/csrc tools/slot_balance.cpp riptide_amd/csrc/plan.cpp -o /tmp/slot_balance
// usage: slot_balance N TSAMP PMIN PMAX BMIN BMAX NW WMAX SCRATCH_MFLOATS
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "plan.hpp"

using namespace rt;

int main(int argc, char** argv)
{
    if (argc < 10) {
        std::fprintf(stderr, "usage: slot_balance N TSAMP PMIN PMAX BMIN BMAX NW WMAX SCRATCH_MFLOATS\n");
        return 2;
    }
    PgramParams prm;
    prm.size = std::strtoull(argv[1], nullptr, 10);
    prm.tsamp = std::atof(argv[2]);
    prm.pmin = std::atof(argv[3]);
    prm.pmax = std::atof(argv[4]);
    prm.bmin = std::strtoull(argv[5], nullptr, 10);
    prm.bmax = std::strtoull(argv[6], nullptr, 10);
    const uint32_t nw = (uint32_t)std::atoi(argv[7]), wmax = (uint32_t)std::atoi(argv[8]);
    const uint64_t budget = (uint64_t)(std::atof(argv[9]) * 1e6);
    PgramPlan pg;
    build_pgram_plan(prm, pg);
    std::vector<FfaXform> xf;
    for (const Step& s : pg.steps) {
        if (!s.rows_eval) continue;
        FfaXform X{};
        X.p = s.bins;
        X.m = s.rows;
        X.rows_eval = s.rows_eval;
        X.rung = s.rung;
        X.src_off = pg.rungs[s.rung].leaf_off;
        X.snr_row = s.out_row;
        X.stdnoise = s.stdnoise;
        xf.push_back(X);
    }
    ExecPlan ex;
    build_exec_plan(xf, true, nw, budget, ex, wmax, 1);
    const double cost[4] = {4.0, 8.0, 5.0, 6.0};   // kSlotOne, kSlotTwo, kSlotPair, kSlotHalf
    double crit = 0, mean = 0, crit_n = 0, mean_n = 0;
    uint64_t steps = 0, kinds[4] = {};
    for (const Launch& L : ex.launches) {
        if (L.smax != 4 && L.smax != 5) continue;
        const int rw = L.rw ? (int)L.rw : merge_rows_per_wave((int)L.smax);
        const int Q = (rw + 1) / 2;
        for (uint32_t k = L.first; k < L.first + L.count; ++k) {
            const ConeItem& it = ex.items[k];
            if (it.pad == kNoBlob || it.levels == 0) continue;
            const uint32_t* w = ex.blob.data() + it.pad;
            for (int lo = 0; lo < (int)it.levels; ++lo) {
                const uint32_t so = w[kHdrSlotOff + lo];
                if (!so) continue;
                const uint32_t ns = w[so];
                double wc[8] = {}, wn[8] = {};
                for (uint32_t g = 0; g < ns; ++g) {
                    const uint32_t wq = (g % kConeWaves) * (uint32_t)Q + g / kConeWaves;
                    const uint32_t sw = w[so + 4 + 4 * wq + 3];
                    const uint32_t kind = sw >> 20;
                    wc[g % 8] += cost[kind];
                    wn[g % 8] += 1;
                    ++kinds[kind];
                }
                crit += *std::max_element(wc, wc + 8);
                crit_n += *std::max_element(wn, wn + 8);
                double s = 0, sn = 0;
                for (int i = 0; i < 8; ++i) s += wc[i], sn += wn[i];
                mean += s / 8;
                mean_n += sn / 8;
                ++steps;
            }
        }
    }
    std::printf("4/5-slot steps %llu  kinds one %llu two %llu pair %llu half %llu\n", (unsigned long long)steps,
                (unsigned long long)kinds[0], (unsigned long long)kinds[1], (unsigned long long)kinds[2],
                (unsigned long long)kinds[3]);
    std::printf("weighted: critical / mean = %.4f   slots: critical / mean = %.4f\n", crit / mean, crit_n / mean_n);
    return 0;
}

// Host-only dump of a periodogram's cone schedule: per launch the pass, slot
// bucket, final/merge-only, units, algorithmic and moved bytes, cells, and
// the unit mix (mode, levels, rows).  Build (host only, no device code):
//   g++ -O2 -std=c++17 -I riptide_amd/csrc tools/sched_dump.cpp riptide_amd/csrc/plan.cpp -o /tmp/sched_dump
// usage: sched_dump N TSAMP PMIN PMAX BMIN BMAX NW WMAX SCRATCH_MFLOATS
#include <cstdio>
#include <cstdlib>
#include <array>
#include <map>
#include <vector>

#include "plan.hpp"

using namespace rt;

int main(int argc, char** argv)
{
    if (argc < 10) {
        std::fprintf(stderr, "usage: sched_dump N TSAMP PMIN PMAX BMIN BMAX NW WMAX SCRATCH_MFLOATS\n");
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
    std::printf("transforms %zu items %zu launches %zu\n", xf.size(), ex.items.size(), ex.launches.size());
    double tot_alg = 0, tot_moved = 0;
    for (size_t i = 0; i < ex.launches.size(); ++i) {
        const Launch& L = ex.launches[i];
        std::map<int, int> lv;
        uint64_t rows = 0, whole = 0;
        for (uint32_t k = L.first; k < L.first + L.count; ++k) {
            const ConeItem& it = ex.items[k];
            lv[it.levels]++;
            rows += it.mode == kModeWhole ? it.node_size : (it.s1 - it.s0);
            whole += it.mode == kModeWhole;
        }
        tot_alg += L.alg_bytes;
        tot_moved += L.moved_bytes;
        std::printf("L%-2zu g%u pass %u smax %u snr %u units %7u whole %7llu out_rows/unit %6.1f alg %.3f GB moved %.3f GB cells %.3f G levels:",
                    i, L.group, L.pass, L.smax, L.snr, L.count, (unsigned long long)whole, (double)rows / L.count,
                    L.alg_bytes / 1e9, L.moved_bytes / 1e9, L.cells / 1e9);
        for (auto& kv : lv) std::printf(" %d:%d", kv.first, kv.second);
        std::printf("\n");
        if (std::getenv("DUMP_DETAIL")) {
            // per (levels, node-size class): units, mean out rows, mean bottom rows (blob), mean transform m
            std::map<std::pair<int,int>, std::array<double,4>> h;
            for (uint32_t k = L.first; k < L.first + L.count; ++k) {
                const ConeItem& it = ex.items[k];
                const int nb = it.pad != kNoBlob ? (int)ex.blob[it.pad + kHdrBottom] : (int)it.node_size;
                int cls = 0;
                while ((1u << cls) < it.node_size) ++cls;
                auto& e = h[{it.levels, cls}];
                e[0] += 1; e[1] += it.mode == kModeWhole ? it.node_size : (it.s1 - it.s0); e[2] += nb; e[3] += ex.xf[it.xform].m;
            }
            for (auto& kv : h)
                std::printf("    L=%d node<=2^%-2d units %7.0f out %6.1f bottom %6.1f (x%.3f) m %8.0f\n", kv.first.first,
                            kv.first.second, kv.second[0], kv.second[1] / kv.second[0], kv.second[2] / kv.second[0],
                            kv.second[2] / kv.second[1], kv.second[3] / kv.second[0]);
        }
    }
    std::printf("total alg %.3f GB moved %.3f GB per trial\n", tot_alg / 1e9, tot_moved / 1e9);
    return 0;
}

// Host tool: LDS merge-read accounting of the cfg2 cone schedule (how many
// ds_read_b32 the kernel issues vs the rows each step actually outputs).
// hipcc -O2 -I riptide_amd/csrc tools/plan_waste.cpp riptide_amd/csrc/plan.cpp -o /tmp/plan_waste
#include <cstdio>
#include <map>
#include <vector>

#include "plan.hpp"

using namespace rt;

int main(int argc, char** argv)
{
    PgramParams a;
    a.size = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1u << 23);
    a.tsamp = argc > 2 ? std::atof(argv[2]) : 256e-6;
    a.pmin = argc > 3 ? std::atof(argv[3]) : 0.1;
    a.pmax = argc > 4 ? std::atof(argv[4]) : 10.0;
    a.bmin = argc > 5 ? std::atoi(argv[5]) : 240;
    a.bmax = argc > 6 ? std::atoi(argv[6]) : 260;
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
    build_exec_plan(xf, true, 6, 1ull << 40, ex);
    double rows_tot = 0, items_tot = 0, noblob = 0, noblob_rows = 0, blob_units = 0;
    double issued = 0, useful = 0, ideal = 0, steps = 0, units = 0;
    std::map<int, double> by_rw_issued, by_rw_useful;
    for (const Launch& L : ex.launches) {
        const int rw = L.rw ? (int)L.rw : merge_rows_per_wave((int)L.smax);
        const int S = slot_count((int)L.smax);
        for (uint32_t i = L.first; i < L.first + L.count; ++i) {
            const ConeItem& it = ex.items[i];
            const uint32_t p = ex.xf[it.xform].p;
            const bool tile = it.mode == kModeTile;
            const int Lv = it.levels;
            auto rows_at = [&](int l) -> int {
                if (it.pad != kNoBlob) return (int)ex.blob[it.pad + l];
                return (int)it.node_size;
            };
            units += 1;
            if (it.pad == kNoBlob) { noblob += 1; noblob_rows += it.node_size; } else blob_units += 1;
            if (it.pad != kNoBlob) {
                const uint32_t* w = ex.blob.data() + it.pad;
                const uint32_t* desc = w + kBlobHeader + 4 * w[24];
                for (int l = Lv - 1; l >= 0;) {
                    const bool two = l >= 1 && (int)L.smax != kPack2 && (tile || (it.node_size >> l) >= 2);
                    const int lo = two ? l - 1 : l;
                    const uint32_t n = w[lo];
                    const uint32_t* d = desc + w[12 + lo];
                    uint32_t items = 0, pairs = 0;
                    for (uint32_t r = 0; r < n;) {
                        const uint32_t a = d[r];
                        if (r + 1 < n && ((a ^ d[r + 1]) & 0xFFFFFu) == 0 && ((a >> 10) & 1023u) != kCarriedRow &&
                            (d[r + 1] >> 20) == ((a >> 20) + 1) % p) {
                            ++pairs;
                            r += 2;
                        } else
                            r += 1;
                        ++items;
                    }
                    const int reads = two ? 4 : 2;
                    rows_tot += (double)n * S * reads;
                    items_tot += (double)items * S * reads;
                    l = lo - 1;
                }
            }
            for (int l = Lv - 1; l >= 0;) {
                const bool two = l >= 1 && (int)L.smax != kPack2 && (tile || (it.node_size >> l) >= 2);
                const int lo = two ? l - 1 : l;
                const int orows = rows_at(lo);
                const int reads = two ? 4 : 2;
                issued += (double)kConeWaves * rw * S * reads;
                useful += (double)orows * S * reads / row_pack((int)L.smax);
                ideal += (double)orows * (p / 64.0) * reads;
                by_rw_issued[rw] += (double)kConeWaves * rw * S * reads;
                by_rw_useful[rw] += (double)orows * S * reads / row_pack((int)L.smax);
                steps += 1;
                l = lo - 1;
            }
        }
    }
    double alg = 0, moved = 0;
    for (const Launch& L : ex.launches) { alg += L.alg_bytes; moved += L.moved_bytes; }
    std::printf("alg GB %.3f moved GB %.3f launches %zu\n", alg / 1e9, moved / 1e9, ex.launches.size());
    std::printf("units %.0f steps %.0f  ds_read issued %.3e useful-rows %.3e ideal-bins %.3e  (useful/issued %.3f)\n",
                units, steps, issued, useful, ideal, useful / issued);
    std::printf("LDS time at 2 clk/read over 256 CUs @2.4GHz: issued %.3f ms, useful %.3f ms\n",
                issued * 2 / 256 / 2.4e9 * 1e3, useful * 2 / 256 / 2.4e9 * 1e3);
    std::printf("units without blob %.0f (avg rows %.1f), with blob %.0f\n", noblob, noblob_rows / (noblob > 0 ? noblob : 1), blob_units);
    std::printf("table units: reads by rows %.3e, by row pairs %.3e (%.3f)\n", rows_tot, items_tot, items_tot / rows_tot);
    for (auto& kv : by_rw_issued)
        std::printf("  rw %2d issued %.3e useful %.3e (%.3f)\n", kv.first, kv.second, by_rw_useful[kv.first],
                    by_rw_useful[kv.first] / kv.second);
}

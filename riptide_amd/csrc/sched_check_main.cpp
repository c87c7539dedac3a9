// Host-only schedule checker, built with AddressSanitizer + UBSan by
// `make -C riptide_amd/csrc asan`: drives the host
// planner and the C ABI's host-only entry points -- rt_periodogram_grid,
// rt_schedule_check, rt_ffa_schedule_check, rt_ladder_check -- which build
// every unit blob, DMA segment table and row-slot table the cone kernel
// trusts.  No device call.  Usage:
//   sched_check pgram N TSAMP PMIN PMAX BMIN BMAX NWIDTHS
//   sched_check ffa ROWS COLS
// Prints one line of results; exit status 0 iff every call returned RT_OK.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "riptide_amd.h"

int main(int argc, char** argv)
{
    if (argc >= 9 && !std::strcmp(argv[1], "pgram")) {
        const size_t n = std::strtoull(argv[2], nullptr, 10);
        const double tsamp = std::atof(argv[3]), pmin = std::atof(argv[4]), pmax = std::atof(argv[5]);
        const size_t bmin = std::strtoull(argv[6], nullptr, 10), bmax = std::strtoull(argv[7], nullptr, 10);
        const size_t nw = std::strtoull(argv[8], nullptr, 10);
        size_t L = 0;
        if (rt_periodogram_length(n, tsamp, pmin, pmax, bmin, bmax, &L)) {
            std::printf("length: %s\n", rt_last_error());
            return 1;
        }
        std::vector<double> periods(L);
        std::vector<uint32_t> foldbins(L);
        if (rt_periodogram_grid(n, tsamp, pmin, pmax, bmin, bmax, periods.data(), foldbins.data())) {
            std::printf("grid: %s\n", rt_last_error());
            return 1;
        }
        uint64_t xf = 0, items = 0, launches = 0, cells = 0;
        double alg = 0, moved = 0;
        if (rt_schedule_check(n, tsamp, nw, pmin, pmax, bmin, bmax, &xf, &items, &launches, &alg, &moved, &cells)) {
            std::printf("schedule: %s\n", rt_last_error());
            return 1;
        }
        int fused = -1;
        uint64_t rungs = 0;
        if (rt_ladder_check(n, tsamp, pmin, pmax, bmin, bmax, &fused, &rungs)) {
            std::printf("ladder: %s\n", rt_last_error());
            return 1;
        }
        std::printf("pgram L=%zu transforms=%llu items=%llu launches=%llu alg=%.6e moved=%.6e fused=%d rungs=%llu\n", L,
                    (unsigned long long)xf, (unsigned long long)items, (unsigned long long)launches, alg, moved, fused,
                    (unsigned long long)rungs);
        return 0;
    }
    if (argc >= 4 && !std::strcmp(argv[1], "ffa")) {
        uint64_t launches = 0;
        if (rt_ffa_schedule_check(std::strtoull(argv[2], nullptr, 10), std::strtoull(argv[3], nullptr, 10), &launches)) {
            std::printf("ffa: %s\n", rt_last_error());
            return 1;
        }
        std::printf("ffa launches=%llu\n", (unsigned long long)launches);
        return 0;
    }
    std::fprintf(stderr, "usage: sched_check pgram N TSAMP PMIN PMAX BMIN BMAX NWIDTHS | ffa ROWS COLS\n");
    return 2;
}

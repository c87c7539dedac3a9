// Host-side planner: periodogram ladder (bit-exact with periodogram.hpp), the
// trial-period grid, and the pass / work-item schedule of the cone kernel.
#pragma once
#include <string>
#include <vector>

#include "common.hpp"

namespace rt {

struct PgramParams {
    size_t size = 0;       // input samples N
    double tsamp = 0, pmin = 0, pmax = 0;
    size_t bmin = 0, bmax = 0;
};

// periodogram.hpp:25-40.  Returns the reference's exception text, or "" if valid.
std::string check_pgram_args(const PgramParams& a);

// downsample.hpp:11-38
size_t downsampled_size(size_t n, double f);
double downsampled_variance(size_t n, double f);

struct Rung {
    double f = 0, tau = 0;
    size_t n = 0;          // downsampled length
    uint64_t leaf_off = 0; // float offset in the per-trial leaf buffer
};

struct Step {              // one (rung, bins) FFA transform
    uint32_t rung = 0, bins = 0, rows = 0, rows_eval = 0;
    float stdnoise = 0;
    uint64_t out_row = 0;  // first grid/S/N row
};

struct PgramPlan {
    PgramParams prm;
    std::vector<Rung> rungs;
    std::vector<Step> steps;
    uint64_t length = 0;       // periodogram_length (periodogram.hpp:63-109)
    uint64_t leaf_floats = 0;  // per-trial leaf buffer (all rungs)
};

// Ladder + steps (periodogram.hpp:135-183).  Arguments must be valid.
void build_pgram_plan(const PgramParams& a, PgramPlan& plan);

// periods[s] / foldbins[s] for all L rows (periodogram.hpp:190-194, in the form
// the reference binary evaluates it: (B*B*tau) / fma(s, -1/(rows-1), B)).
void fill_grid(const PgramPlan& plan, double* periods, uint32_t* foldbins);

struct Launch {
    uint32_t first = 0, count = 0;   // item range
    uint32_t group = 0, pass = 0;
    uint32_t smax = 0;               // cone kernel variant: merge_slots() of every transform in the launch
    uint32_t rw = 0;                 // register rows per wave of the variant (0: merge_rows_per_wave(smax))
    uint32_t wide_snr = 0;           // final units whose S/N reads wide widths as plain LDS windows (WIDE variant)
    uint32_t snr = 0;                // 1: every unit ends in the fused S/N (a final pass); 0: none does
    double alg_bytes = 0;            // 4mp read + (4mp | 4*rows_eval*W) write
    double moved_bytes = 0;          // bytes the items actually read + write (cone overlap incl.)
    uint64_t cells = 0;              // sum m*p of the transforms in this launch
};

struct ExecPlan {
    std::vector<FfaXform> xf;
    std::vector<ConeItem> items;     // tile items: ConeItem::pad = word offset of their blob
    std::vector<Launch> launches;
    std::vector<uint32_t> blob;      // host-built metadata of every tile item (build_tile_blob)
    uint64_t scratch_floats = 0;     // per ping/pong buffer, per trial (all banks)
    uint32_t max_passes = 0;
    // scratch banks: 2 = odd transform groups use a second copy of the
    // scratch (offset bank_floats), so two groups can run at once on two
    // streams (capi.cpp run_cone_launches: co-scheduling)
    uint32_t banks = 1;
    uint64_t bank_floats = 0;
    uint32_t groups = 0;
};

// Tile-unit metadata built on the host once per plan (the cone kernel reads
// it, never recomputes it): the dependency cone's range tree flattened into
// rows per level, the row-descriptor table of every level (head row | tail
// row << 10 | roll shift << 20, transforms.hpp:13-27 restated per row), the
// LDS float offset of every bottom row in the fill layout, the row-slot table
// of every merge step (slot_rw > 0: the launch's register rows per wave, see
// kSlotPair) and the LDS DMA segments of the bottom level.  Blob layout
// (uint32 words, 16-byte aligned; common.hpp kHdr*):
//   [0, 12)  rows of levels 0..L        [12, 24) first descriptor of each level
//   [24] DMA segments  [25] descriptor entries  [26] bottom rows  [27] slot words
//   [28] word offset of the segments    [32, 44) slot table of each level (0: none)
//   [48, ...) descriptor table (entries words), bottom-row offsets, slot
//             tables (each: slots, then one word per slot)  -- the LDS part
//   [segments offset, + 4 segments)  per segment (one LDS-DMA wave
//             instruction): first LDS chunk, chunks (<= 64), first source
//             chunk (16 bytes) in the transform block, 0
// packed (kPack2 units): instead of row-slot tables, every two-level step
// gets a table of its output rows pre-resolved (2 words per row: the four
// source rows, the three rolls) and the descriptor table keeps only the
// levels single steps read.
// Resolved slot tables (4/5-slot variants, resolved_slots): per slot two
// 16-byte entries (row A, row B) of source-row LDS offsets, rolls and the
// slot word; no descriptor table.
void build_tile_blob(const ConeItem& it, uint32_t p, int slot_rw, int smax, std::vector<uint32_t>& out);

// Schedule a list of transforms (p, m, rows_eval, src_off, snr_row, stdnoise
// filled in by the caller).  With snr_epilogue the last pass of every
// transform writes S/N rows; otherwise it writes the transform into `ping`.
// Transforms are grouped so that each group's scratch fits scratch_budget
// floats per buffer; a group's passes are consecutive launches.  max_width
// (the widest boxcar, 0 = unknown) caps final tiles for the S/N's wide stride.
// banks = 2: odd groups' scratch in a second bank (co-scheduling of two groups).
// Within a group, every merge-only launch precedes every final (fused S/N) one.
void build_exec_plan(const std::vector<FfaXform>& xforms, bool snr_epilogue, uint32_t num_widths,
                     uint64_t scratch_budget, ExecPlan& out, uint32_t max_width = 0, uint32_t banks = 1);

// Schedule invariants (every item fits its LDS / register budget and stays
// inside its node, the final pass of every transform covers rows [0, m) once,
// every transform block stays below the 2 GiB range of a 32-bit buffer
// resource).  Throws std::runtime_error on a violation; build_exec_plan runs
// it on every plan it returns, so a kernel never receives an invalid unit.
void validate_exec_plan(const ExecPlan& ex, bool snr_epilogue);

// Byte size limit of one transform block (m x p floats): the cone kernel
// addresses a block through a buffer resource with a 32-bit byte count and
// sends dropped lanes to offset 2^31.
constexpr uint64_t kMaxBlockBytes = 1ull << 31;

// Dependency-cone footprint of one tile (host mirror of the device range tree).
struct ConeNeed { int max_rows = 0; int max_floats = 0; int ranges = 0; int rows_bottom = 0; int runs_bottom = 0; int entries = 0; bool degenerate = false; };
ConeNeed cone_need(uint32_t node_size, uint32_t s0, uint32_t s1, int levels, uint32_t p);

}  // namespace rt

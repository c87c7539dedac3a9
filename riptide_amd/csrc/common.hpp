// Shared host/device definitions of the MI355X FFA periodogram engine.
//
// Data model: a periodogram is a ladder of rungs (downsampling
// factors f); each rung contributes one FFA transform per phase-bin count
// B in [bins_min, bstop].  A transform of m rows x p (= B) columns is evaluated
// as a sequence of *passes*; each pass is one launch of the cone kernel over a
// list of work items (one workgroup each).
//
//   pass 0  ("whole" items): every node of the FFA split tree at depth d_b is
//           small enough (<= C rows) to be transformed entirely in LDS, from
//           the leaves (rows of the downsampled series) up.
//   pass k  ("tile" items):  K consecutive output rows of a node at depth d,
//           computed from the rows they depend on L levels below (their
//           dependency cone), again entirely in LDS.
//
// The last pass of a transform fuses the boxcar S/N scan (snr.hpp:37-65) on the
// rows it produced, so the transform output never returns to HBM.
#pragma once
#include <cstddef>
#include <cstdint>

#if defined(__HIPCC__)
#define RT_HD __host__ __device__
#else
#define RT_HD
#endif

namespace rt {

// ---- cone kernel geometry (gfx950: 160 KiB LDS per CU): two 512-thread
// workgroups per CU (8 waves each, <= 128 VGPRs), one 71 KiB level buffer
// each; the CU's other workgroup fills one's fill and startup latency.  (The
// one-16-wave-workgroup double-buffered layout and the 3- / 4-workgroup
// layouts were measured slower: DESIGN.md section 5.)  The merged levels are
// dense rows (stride p).
constexpr int kConeWgsPerCu = 2;
constexpr int kConeBlock = 512;
static_assert(kConeBlock % 64 == 0, "whole waves");
constexpr int kConeWaves = kConeBlock / 64;
constexpr int kConeWavesPerSimd = kConeWgsPerCu * kConeWaves / 4;
constexpr int kLdsBufFloats = 18176;        // one level buffer: a unit's fill (16-byte chunks, runs per range)
constexpr int kLdsDataFloats = kLdsBufFloats - 256;   // rows x p of any level (the rest: per-range 16-byte phase slack)
constexpr int kLdsPadFloats = 128;          // slack read (never used) by the unused slots of the last row
constexpr int kMaxRows = 384;               // rows per level (row-offset table, descriptors)
constexpr int kDescEntries = 1024;          // row-descriptor table (all levels of a unit)
constexpr int kMaxTileLevels = 6;           // L for tile items
constexpr int kMaxLevels = 11;              // merge levels of any unit (whole units: ceil(log2(kMaxRows)))
constexpr int kMaxRanges = (1 << (kMaxTileLevels + 1)) - 1;
constexpr int kMaxWidths = 32;              // boxcar widths handled by the fused S/N epilogue
constexpr int kSnrChunk = 17;               // S/N epilogue: columns per lane held in registers
// S/N epilogue (ffa_kernels.hip snr_rows): widths <= kSnrWin from a
// register window; chunk columns per lane of the register-window path
constexpr int kSnrWin = 12;
constexpr int kSnrMaxChunk = 17;
// Widths past the register window as plain LDS windows: a final level whose
// row stride holds the wrapped prefix c[p + e] = c[e] + sum for e < wmax
// after each row, so every lane's column j0 + t + w (t < its chunk) is a
// plain read (the planner caps final tiles so their rows fit at this stride:
// plan.cpp final_tile_cap).
RT_HD inline int snr_wide_stride(int p, int wmax)
{
    return p + (wmax > kSnrMaxChunk ? wmax : kSnrMaxChunk);
}
RT_HD inline bool snr_wide_ok(int p, int q, int wmax)
{
    return wmax > kSnrWin && wmax < p && q >= snr_wide_stride(p, wmax);
}
// S/N lane-group size G of a row of p bins: the smallest power of two >= 8
// whose chunks ((p + G - 1) / G, made odd) fit kSnrMaxChunk columns.  The
// wide path runs in the 16-lane groups (p = 137-272).
RT_HD constexpr int snr_group(int p)
{
    int G = 8;
    while (G < 64 && ((((p + G - 1) / G) | 1) > kSnrMaxChunk)) G <<= 1;
    return G;
}
// Segmented S/N (ffa_kernels.hip snr_segments): a final level of <= 64 rows
// of 240-264 bins, widths <= 9, one row per lane, each of the 8 waves a
// segment of kSnrSegCols columns.  Row r lies in an LDS slot of
// kSnrSegStride floats (odd: 64 rows on distinct banks) at offset
// 8 kSnrSegCols - p, so the first segment starts at the slot start; the
// segment sums are exchanged through kSnrSegExch floats at the end of the
// level buffer (past kLdsDataFloats: the fill slack is dead by then).
constexpr int kSnrSegCols = 33;
constexpr int kSnrSegWmax = 9;
constexpr int kSnrSegRows = 64;
constexpr int kSnrSegStride = 8 * kSnrSegCols + 1;
constexpr int kSnrSegExch = 2 * 64 * 8;
static_assert(kSnrSegRows * kSnrSegStride <= kLdsDataFloats, "segmented S/N rows");
static_assert(kSnrSegRows * kSnrSegStride + kSnrSegExch <= kLdsBufFloats, "segmented S/N exchange area");
RT_HD inline bool snr_seg_ok(int p, int wmax, int rows)
{
    return p >= 8 * kSnrSegCols - 24 && p <= 8 * kSnrSegCols && wmax >= 1 && wmax <= kSnrSegWmax && rows >= 1 &&
           rows <= kSnrSegRows;
}
constexpr int kStageRegs = 45 * 8 / kConeWaves;   // merge: staged values per lane (rows x slots)
constexpr int kMaxSlots = 45;               // merge: 64-bin slots per row (p <= 2880)
constexpr int kMaxRowsPerWave = 24;         // merge: staged rows per wave
// header words of a unit's host-built blob (plan.hpp build_tile_blob); a
// unit without one (a whole unit too large for the descriptor table) has
// UnitDesc::pad = kNoBlob.  kCarriedRow: the tail-row field of a size-1 node
// carried unchanged.
constexpr int kBlobHeader = 48;
// header words: rows of levels 0..L at [0, 12), first descriptor of each
// level at [12, 24), then the counts, then the row-slot table of each merge
// step's output level at [32, 44) (0: no table)
enum : int {
    kHdrRows = 0, kHdrDesc = 12, kHdrRuns = 24, kHdrEntries = 25, kHdrBottom = 26, kHdrSlotWords = 27,
    kHdrRunOff = 28, kHdrFill = 29, kHdrZero = 30, kHdrSlotOff = 32
};
// kHdrZero: LDS float offset of a whole unit's zero row (0: none).  A 4/5-slot
// whole unit with an even number of levels fuses every step, its deepest one
// included, although that step's middle level holds carried size-1 nodes: a
// carried node's missing tail operand reads a row of -0.0 (x + (-0.0) == x,
// the reference's copy), laid after the unit's fill -- three LDS passes
// instead of four (single, fused, fused, single).  Only the deepest step reads
// it; a final unit's output level may cover it, so final units rewrite it
// before every trial.
// row slots (merge steps of units with a blob, SMAX <= 5): a wave's register
// rows 2q, 2q + 1 hold slot q: one row, two independent rows, or a row pair
// r, r + 1 with the same head and tail rows and roll shifts s, s + 1 (the
// second row's tail term is the first's shifted by one bin).  Slot word:
// row A | row B << 10 | kind << 20.
enum : uint32_t { kSlotOne = 0, kSlotTwo = 1, kSlotPair = 2, kSlotHalf = 3 };
// kSlotHalf: rows r, r + 1 with the same head row (not a pair: their tails or
// shifts differ -- an odd-sized node's consecutive outputs), so the head term
// (the level-l+1 head row H', or H for a single step) is computed once for
// both and only row B's tail term is read (RT_SLOT_HALF: the planner emits
// them; the kernel always runs them)
constexpr int kSlotWords = 544;             // LDS area of a unit's slot tables
// 4/5-slot variants (p = 193-320, rows <= 72 per unit): slot tables with
// every row resolved (build_tile_blob), 16 bytes per row: source-row LDS
// offsets (16 bits each), the three rolls (10 bits each, | carried << 30 for
// single steps) and the slot word
RT_HD constexpr bool resolved_slots(int smax) { return smax == 4 || smax == 5; }
constexpr int kAuxMetaWords = kBlobHeader + kDescEntries + kMaxRows + kSlotWords;   // the metadata area
// 4-slot roll table (ffa_kernels.hip row_terms_lut): 2 words per entry
// x < 256 + 64 at the end of the metadata area, which it extends by kLutPad
// words (the workgroup's LDS stays inside the same 512-byte granule); every
// 4-slot row-slot unit's blob LDS part must end at or before kLut4Off
constexpr int kLutPad = 64;
constexpr int kLut4Words = 2 * (256 + 64);
constexpr int kLut4Off = kAuxMetaWords + kLutPad - kLut4Words;
constexpr uint32_t kNoBlob = 0xFFFFFFFFu;
constexpr uint32_t kCarriedRow = 1023;
// 16-byte chunks of a unit's LDS DMA fill (setup_unit): a whole unit's block
// of n*p floats at 16-byte phase <= 3, or a tile's ranges, each a run at its
// own phase (<= 2^L runs); the planner keeps every unit within a buffer.
RT_HD inline int fill_chunks_bound(int n, int p, int runs) { return (n * p + 6 * runs + 3) >> 2; }
// Units of the kPack2 variant (p <= 32: short rows leave most of the level
// buffer free) keep their blob's LDS part (header, descriptors, bottom-row
// offsets; no slot tables) at the end of their own level buffer instead of
// the fixed metadata area, so the descriptor table may hold every level of
// a 384-row unit.
RT_HD inline int pack_blob_words(int entries, int nb) { return (kBlobHeader + entries + nb + 2 * kMaxLevels + 4) & ~3; }

// Merge variant for rows of p phase bins: slots per row rounded up to an
// instantiated width (1..5, 8, 11, 16, 22, 45), or kPack2 for p <= 32 (short rows:
// (row, 8-bin segment) tasks, ffa_kernels.hip merge_step_tasks); 0 if p is
// too wide for the LDS engine.  The value is the cone kernel's template
// argument and launch bucket.
constexpr int kPack2 = 64;
RT_HD inline int merge_slots(uint32_t p)
{
    if (p <= 32) return kPack2;
    if (p == 0) return 1;
    const int s = (int)((p + 63) / 64);
    if (s <= 5) return s;
    if (s <= 8) return 8;
    if (s <= 11) return 11;
    if (s <= 16) return 16;
    if (s <= 22) return 22;
    if (s <= kMaxSlots) return kMaxSlots;
    return 0;
}

// Row stride of the merge levels above the fill in the short-row variant
// (kPack2, ffa_kernels.hip merge_step_tasks).  The interleaved tasks (lane
// (row, segment s) takes bins s + segs*k, k < 8) write up to 8*segs bins per
// row, so the stride is >= 8*segs; for 16 <= p <= 32 it is the stride with
// the fewest LDS bank conflicts of those steps' reads over the cfg4
// schedule (a host simulation of every task address; 1.05-1.34 x the
// conflict-free cycles against 1.08-2.25 x at the odd stride p | 1).
RT_HD inline int pack_stride(int p)
{
    if (p < 8) return p;
    if (p < 16) return p <= 8 ? 9 : 17;
    if (p <= 32)
        return p == 16 ? 34 : p < 20 ? 35 : p < 25 ? 36 : p < 28 ? 37 : p == 28 ? 36 : p == 29 ? 37 : 38;
    return p | 1;
}
// 64-lane slots per register row of a merge variant, and rows per slot
RT_HD constexpr int slot_count(int smax) { return smax == kPack2 ? 1 : smax; }
RT_HD constexpr int row_pack(int smax) { return smax == kPack2 ? 2 : 1; }

// Register rows per wave the merge stages for a variant (register budget);
// each register row holds row_pack(smax) output rows.  The 4-slot variant
// stages 9: its LDS capacity at p >= 240 (9 x 8 waves = 72 >= 16128 / 240).
constexpr int kRw4 = (72 + kConeWaves - 1) / kConeWaves;
RT_HD constexpr int merge_rows_per_wave(int smax)
{
    return smax == 4
               ? kRw4
               : (kStageRegs / slot_count(smax) < 1
                      ? 1
                      : (kStageRegs / slot_count(smax) < kMaxRowsPerWave ? kStageRegs / slot_count(smax)
                                                                         : kMaxRowsPerWave));
}

// Row capacity of one cone work unit for p phase bins run by the kernel
// variant smax (merge_slots(p), or a wider slot width): the level buffer, and
// the register staging of a level (merge_rows_per_wave(smax) register rows
// of row_pack(smax) rows per wave).
RT_HD inline int lds_row_capacity(uint32_t p, int smax)
{
    if (!smax || p == 0) return 0;
    int c = kLdsDataFloats / (int)p;
    const int stage = kConeWaves * merge_rows_per_wave(smax) * row_pack(smax);
    if (stage < c) c = stage;
    return c < kMaxRows ? c : kMaxRows;
}

RT_HD inline int lds_row_capacity(uint32_t p) { return lds_row_capacity(p, merge_slots(p)); }

// One FFA transform of a plan ((rung, bins) step of periodogram.hpp:153-199).
struct FfaXform {
    uint32_t p;          // phase bins (= columns)
    uint32_t m;          // rows (= n / p)
    uint32_t rows_eval;  // rows whose S/N is evaluated (periodogram.hpp:183)
    uint32_t rung;
    uint64_t src_off;    // float offset of the leaf rows in the per-trial leaf buffer
    uint64_t buf_off;    // float offset of the scratch rows in ping/pong
    uint64_t snr_row;    // first S/N output row (prefix sum of rows_eval)
    float stdnoise;      // periodogram.hpp:181
    uint32_t pad;
};
static_assert(sizeof(FfaXform) == 48, "FfaXform layout");

enum : uint8_t { kModeWhole = 0, kModeTile = 1 };
// RT_STAMPS diagnostic builds: one record per work unit of kStampRecWords
// words: hw id | xcc << 32, kStampMarks s_memtime marks (start, setup done,
// fill issued, descriptors built, fill landed, merge done, end), shape bits.
constexpr int kStampMarks = 16;   // + S/N pass 0: prefix, barrier, window, end; + unit_begin: view, header, DMA issued;
                                   // + workgroup entry / exit on the device-wide 100 MHz clock
constexpr int kStampRecWords = kStampMarks + 2;
constexpr uint64_t kTimelineCap = 1u << 23;
// cone kernel feature bits (ConeArgs::flags)
enum : uint32_t {
    kConeStoreFromRegs = 1u,   // non-final passes store the output level straight from registers
    kConeFuse2 = 2u,           // two merge levels per LDS round trip where no level holds size-1 nodes
    kConeSnrStride = 4u,       // final passes keep their output rows at a bank-friendly stride for the S/N
    kConeSnrSeg = 8u,          // final passes of 240-264-bin rows with widths <= 9: the segmented S/N (snr_segments)
    kConeDiagNoSnr = 1u << 30, // diagnostics only (wrong results): skip the S/N epilogue
    kConeDiagNoMerge = 1u << 29, // diagnostics only (wrong results): skip the merge levels
    kConeDiagNoWrite = 1u << 28, // diagnostics only (wrong results): skip the level write-back
    kConeDiagNoBarrier = 1u << 27, // diagnostics only (wrong results): no barriers between merge levels
    kConeDiagNoLand = 1u << 26,  // diagnostics only (wrong results): fill loads issued but not landed in LDS
    kConeDiagNoDesc = 1u << 25,  // diagnostics only (wrong results): no descriptor table
    kConeDiagNoFill = 1u << 23,  // diagnostics only (wrong results): metadata DMA only, no bottom-level fill
    kConeDefaultFeatures = 15u  // every feature bit above
};
enum : uint8_t { kSelLeaves = 0, kSelPing = 1, kSelPong = 2, kSelSnr = 3 };

// One workgroup of one pass.
struct ConeItem {
    uint32_t xform;
    uint32_t node_start;  // first row (within the transform) of the target node
    uint32_t node_size;   // rows of the target node
    uint32_t s0, s1;      // output tile [s0, s1) in node-local rows
    uint8_t levels;       // merge levels evaluated by this item
    uint8_t mode;         // kModeWhole / kModeTile
    uint8_t src;          // kSelLeaves / kSelPing / kSelPong
    uint8_t dst;          // kSelPing / kSelPong / kSelSnr
    uint32_t pad;
};
static_assert(sizeof(ConeItem) == 28, "ConeItem layout");

// Device form of one work item: the item and its transform in one 64-byte
// record (a single scalar load per workgroup).
struct UnitDesc {
    uint32_t node_start, node_size, s0, s1;
    uint32_t p, m, rows_eval;
    float stdnoise;
    uint64_t src_off, buf_off, snr_row;
    uint8_t levels, mode, src, dst;
    uint32_t pad;         // word offset of the unit's blob in ConeArgs::blob (kNoBlob: none)
    // the blob's header counts (kHdrRuns .. kHdrRunOff), so the kernel issues
    // the unit's DMA after one scalar load instead of a dependent chain
    uint32_t nruns, entries, nb, slot_words, run_off;
    uint32_t fill_chunks;  // 16-byte chunks of the bottom-level fill
    uint32_t zero_row;     // the blob's kHdrZero: LDS float offset of the unit's -0.0 row (0: none)
    uint32_t pad2;
};
static_assert(sizeof(UnitDesc) == 96, "UnitDesc layout");

// Arguments of one cone-kernel launch.  Per-trial strides are in floats.
struct ConeArgs {
    const UnitDesc* items;
    uint32_t num_items;
    uint32_t num_widths;
    const float* leaves;
    uint64_t leaves_stride;
    float* ping;
    float* pong;
    uint64_t buf_stride;
    float* snr;
    uint64_t snr_stride;
    const uint32_t* widths;  // boxcar widths (bins), device array of num_widths
    int* error_flag;      // set non-zero if a work item violates the LDS budget
    const uint32_t* blob; // host-built tile-unit metadata (plan.hpp build_tile_blob); UnitDesc::pad = word offset
    unsigned long long* stamps;   // RT_STAMPS diagnostic builds only: per-phase cycles
    uint32_t batch;       // trials of the launch
    uint32_t flags;       // kCone* feature bits (A/B experiments; default all set)
    // trials per workgroup (0 = 1): workgroup b runs item b / G for the trials
    // (b % G) * T .. + T - 1 of the batch (G = ceil(batch / T)), one after
    // the other in the same LDS: the item's record, blob (descriptors, slot
    // tables) and roll table are loaded once for all T trials, and a merge-
    // only unit issues the next trial's fill before storing the current one
    uint32_t trials_per_wg;
};
constexpr uint32_t kConeTrialsPerWg = 16;  // default trials per workgroup (capi.cpp cone_trials_per_wg)
// workgroups per item of a cone launch
RT_HD inline uint32_t cone_trial_groups(uint32_t batch, uint32_t tpw)
{
    const uint32_t t = tpw ? tpw : 1u;
    return (batch + t - 1) / t;
}

// Merge index of the FFA recursion (transforms.hpp:17-22): the reference build
// evaluates (size_t)(k * s + 0.5f) with k = (child_rows - 1.0f) / (rows - 1.0f)
// in float32; the fused and unfused forms agree for every rows < 2e5
// (tests/test_oracle_golden.py::test_ffa2_bit_exact).  The fused form is used.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t merge_index(float k, uint32_t s)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_fmaf(k, (float)s, 0.5f);
#else
    return (uint32_t)__builtin_fmaf(k, (float)s, 0.5f);
#endif
}

#if defined(__HIPCC__)
__host__ __device__
#endif
inline float merge_coef(uint32_t child_rows, uint32_t rows)
{
    return ((float)child_rows - 1.0f) / ((float)rows - 1.0f);
}

}  // namespace rt

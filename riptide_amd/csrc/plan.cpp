// Host planner.  Compiled with -ffp-contract=off -mfma: every floating-point
// expression is evaluated as written, and the one FMA the reference binary
// emits (the period grid) is requested explicitly.
#include "plan.hpp"

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <stdexcept>
#include <string>

namespace rt {

std::string check_pgram_args(const PgramParams& a)
{
    // periodogram.hpp:25-40 (same order, same messages)
    if (!(a.tsamp > 0)) return "tsamp must be > 0";
    if (!(a.pmin > 0)) return "period_min must be > 0";
    if (!(a.pmax > a.pmin)) return "period_max must be > period_min";
    if (!(a.bmin > 1)) return "bins_min must be > 1";
    if (!(a.bmax >= a.bmin)) return "bins_max must be >= bins_min";
    if (!(a.pmin >= a.tsamp * (double)a.bmin)) return "Must have: period_min >= tsamp * bins_min ";
    return "";
}

size_t downsampled_size(size_t n, double f)
{
    return (size_t)std::floor((double)n / f);
}

double downsampled_variance(size_t n, double f)
{
    const double k = std::floor(f);
    const double r = f - k;
    const double x = (double)downsampled_size(n, f) * r;
    if (x > 1.0) return f - 1.0 / 3.0;
    return (k - 1.0) * (k - 1.0) + 2.0 / 3.0 * (x * x) - x + 1.0;
}

static size_t ceilshift(size_t rows, size_t cols, double pmax)
{
    // periodogram.hpp:54-57
    return (size_t)std::ceil((double)cols * ((double)rows - 1.0) * (1.0 - (double)cols / pmax));
}

void build_pgram_plan(const PgramParams& a, PgramPlan& plan)
{
    plan = PgramPlan();
    plan.prm = a;
    const double ds_ini = a.pmin / (a.tsamp * (double)a.bmin);
    const double ds_geo = ((double)a.bmax + 1.0) / (double)a.bmin;
    const size_t nds = (size_t)std::ceil(std::log(a.pmax / a.pmin) / std::log(ds_geo));
    uint64_t leaf = 0, row = 0;
    for (size_t ids = 0; ids < nds; ++ids) {
        Rung r;
        r.f = ds_ini * std::pow(ds_geo, (double)ids);
        r.tau = r.f * a.tsamp;
        r.n = downsampled_size(a.size, r.f);
        r.leaf_off = leaf;
        const double pmax_samples = a.pmax / r.tau;
        size_t bstop = std::min(a.bmax, r.n);
        bstop = std::min(bstop, (size_t)pmax_samples);
        const uint32_t rung_index = (uint32_t)plan.rungs.size();
        bool used = false;
        for (size_t bins = a.bmin; bins <= bstop; ++bins) {
            Step s;
            s.rung = rung_index;
            s.bins = (uint32_t)bins;
            s.rows = (uint32_t)(r.n / bins);
            s.stdnoise = (float)std::sqrt((double)s.rows * downsampled_variance(a.size, r.f));
            const double pceil = std::min(pmax_samples, (double)bins + 1.0);
            s.rows_eval = (uint32_t)std::min((size_t)s.rows, ceilshift(s.rows, bins, pceil));
            s.out_row = row;
            row += s.rows_eval;
            plan.steps.push_back(s);
            used = true;
        }
        plan.rungs.push_back(r);
        if (used) leaf += (r.n + 3) & ~(uint64_t)3;   // 16-byte aligned rungs
    }
    plan.length = row;
    plan.leaf_floats = leaf;
}

void fill_grid(const PgramPlan& plan, double* periods, uint32_t* foldbins)
{
    for (const Step& s : plan.steps) {
        const double tau = plan.rungs[s.rung].tau;
        const uint64_t B = s.bins;
        const double num = (double)(B * B) * tau;
        const double r = -1.0 / ((double)s.rows - 1.0);
        for (uint32_t i = 0; i < s.rows_eval; ++i) {
            periods[s.out_row + i] = num / std::fma((double)i, r, (double)B);
            foldbins[s.out_row + i] = (uint32_t)B;
        }
    }
}

// ---------------------------------------------------------------------------
// Pass schedule
// ---------------------------------------------------------------------------
static int ceil_log2(uint32_t s)
{
    int l = 0;
    while ((1u << l) < s) ++l;
    return l;
}

struct Node { uint32_t start, size; };

static void nodes_at_depth(uint32_t m, int depth, std::vector<Node>& out)
{
    out.clear();
    out.push_back({0, m});
    for (int d = 0; d < depth; ++d) {
        std::vector<Node> nxt;
        nxt.reserve(out.size() * 2);
        for (const Node& n : out) {
            if (n.size <= 1) { nxt.push_back(n); continue; }
            const uint32_t h = n.size >> 1;
            nxt.push_back({n.start, h});
            nxt.push_back({n.start + h, n.size - h});
        }
        out.swap(nxt);
    }
}

ConeNeed cone_need(uint32_t node_size, uint32_t s0, uint32_t s1, int levels, uint32_t p)
{
    struct R { uint32_t size, lo, hi; };
    std::vector<R> cur{{node_size, s0, s1 - 1}}, nxt;
    ConeNeed need;
    auto account = [&](const std::vector<R>& lv) {
        int rows = 0;
        for (const R& r : lv) rows += (int)(r.hi - r.lo + 1);
        need.entries += need.rows_bottom; // descriptors of the level above the one accounted now
        need.rows_bottom = rows;          // the last level accounted is the cone's bottom
        need.runs_bottom = (int)lv.size();
        need.max_rows = std::max(need.max_rows, rows);
        need.max_floats = std::max(need.max_floats, rows * (int)p);
        need.ranges += (int)lv.size();
    };
    account(cur);
    for (int l = 0; l < levels; ++l) {
        nxt.clear();
        for (const R& r : cur) {
            // the device range tree assumes 2^l ranges at level l: every node
            // that is merged has >= 2 rows
            if (r.size <= 1) {
                need.degenerate = true;
                nxt.push_back(r);
                continue;
            }
            const uint32_t sh = r.size >> 1, st = r.size - sh;
            const float kh = merge_coef(sh, r.size), kt = merge_coef(st, r.size);
            nxt.push_back({sh, merge_index(kh, r.lo), merge_index(kh, r.hi)});
            nxt.push_back({st, merge_index(kt, r.lo), merge_index(kt, r.hi)});
        }
        cur.swap(nxt);
        account(cur);
    }
    return need;
}

static bool fits(const ConeNeed& n, uint32_t p, int smax)
{
    if (n.degenerate || n.max_rows > lds_row_capacity(p, smax) || n.ranges > kMaxRanges) return false;
    const int fill = 4 * fill_chunks_bound(n.rows_bottom, (int)p, n.runs_bottom);
    if (smax == kPack2)   // the blob at the end of the level buffer (pack_blob_words)
        return std::max(fill, n.max_rows * pack_stride((int)p)) + pack_blob_words(n.entries, n.rows_bottom) <=
               kLdsBufFloats;
    return n.max_floats <= kLdsDataFloats && fill <= kLdsBufFloats && n.entries <= kDescEntries;
}

// Per-transform schedule: list of passes, each a list of (node, tile, levels).
struct PassItems { std::vector<ConeItem> items; double read = 0, written = 0; };

// Tile-level cost model: a pass costs C / (C - cone overhead) merge units plus
// pass_weight() for its HBM round trip and unit setup (RIPTIDE_AMD_PASS_WEIGHT).
// Measured (cfg2, ms per trial): weight 1 -> 11.57, 20 -> 11.47, 100 -> 11.43:
// fewer passes win even at a larger cone overhead, so the default is 100.
static double pass_weight()
{
    if (const char* e = std::getenv("RIPTIDE_AMD_PASS_WEIGHT")) {
        const double v = std::atof(e);
        if (v >= 0) return v;
    }
    return 100.0;
}

// final_kmax: output rows per final-pass tile at most (the wide S/N stride,
// snr_wide_stride); 0 = no cap.
static void plan_transform(const FfaXform& X, uint32_t xi, int smax, uint32_t final_kmax, std::vector<PassItems>& passes)
{
    passes.clear();
    const uint32_t m = X.m, p = X.p;
    const int C = lds_row_capacity(p, smax);
    if (C < 3) throw std::invalid_argument("phase bins too large for the LDS cone kernel");
    // bottom depth: every node at depth db transforms whole in LDS
    int db = 0;
    while (((uint64_t)m + (1ull << db) - 1) >> db > (uint64_t)C) ++db;
    std::vector<Node> nodes;
    nodes_at_depth(m, db, nodes);
    PassItems bottom;
    for (const Node& n : nodes) {
        ConeItem it{};
        it.xform = xi;
        it.node_start = n.start;
        it.node_size = n.size;
        it.s0 = 0;
        it.s1 = n.size;
        it.levels = (uint8_t)ceil_log2(n.size);
        it.mode = kModeWhole;
        bottom.items.push_back(it);
        bottom.read += 4.0 * n.size * p;
        bottom.written += 4.0 * n.size * p;
    }
    passes.push_back(std::move(bottom));
    if (db == 0) return;

    // upper levels: db merge levels in passes of L (cost model: cone overhead vs passes)
    int bestL = 1;
    double best = 1e300;
    for (int L = 1; L <= kMaxTileLevels; ++L) {
        const int extra = 2 << L;
        if (extra + 1 >= C) break;
        const int npass = (db + L - 1) / L;
        const double cost = npass * ((double)C / (double)(C - extra) + pass_weight());
        if (cost < best - 1e-9) { best = cost; bestL = L; }
    }
    const int npass = (db + bestL - 1) / bestL;
    // split db levels as evenly as possible; deeper passes first
    std::vector<int> lv(npass, db / npass);
    for (int i = 0; i < db % npass; ++i) lv[i] += 1;
    int depth_below = db;   // depth whose rows the next pass reads
    for (int k = 0; k < npass; ++k) {
        const int L = lv[k];
        const int dtop = depth_below - L;
        nodes_at_depth(m, dtop, nodes);
        PassItems pass;
        const int guess = std::max(1, C - (2 << L) - 2);
        const uint32_t kmax = k == npass - 1 && final_kmax ? final_kmax : ~0u;
        for (const Node& n : nodes) {
            uint32_t s0 = 0;
            while (s0 < n.size) {
                uint32_t K = std::min<uint32_t>(std::min<uint32_t>((uint32_t)guess, kmax), n.size - s0);
                ConeNeed need = cone_need(n.size, s0, s0 + K, L, p);
                while (K > 1 && !fits(need, p, smax)) {
                    K -= std::max<uint32_t>(1, K / 32);
                    need = cone_need(n.size, s0, s0 + K, L, p);
                }
                if (!fits(need, p, smax)) throw std::invalid_argument("cone tile does not fit in LDS");
                while (s0 + K < n.size && K < kmax) {
                    ConeNeed nn = cone_need(n.size, s0, s0 + K + 1, L, p);
                    if (!fits(nn, p, smax)) break;
                    need = nn;
                    ++K;
                }
                ConeItem it{};
                it.xform = xi;
                it.node_start = n.start;
                it.node_size = n.size;
                it.s0 = s0;
                it.s1 = s0 + K;
                it.levels = (uint8_t)L;
                it.mode = kModeTile;
                pass.items.push_back(it);
                // rows read at the cone bottom (upper bound: max level) + rows written
                pass.read += 4.0 * need.max_rows * p;
                pass.written += 4.0 * K * p;
                s0 += K;
            }
        }
        passes.push_back(std::move(pass));
        depth_below = dtop;
    }
}

// Relative cost of a work item: floats through LDS (bottom rows x p) per merge
// level, plus the load/store.
static double item_cost(const ConeItem& it, const FfaXform& X)
{
    const double rows = it.mode == kModeTile ? (double)(it.s1 - it.s0) + (double)(2u << it.levels)
                                             : (double)it.node_size;
    return rows * (double)X.p * ((double)it.levels + 2.0);
}

// Output rows per final tile that leave room for the wide S/N stride (widths
// past the S/N register window read as plain LDS windows, common.hpp
// snr_wide_stride), or 0 (no cap: no such widths, or the variant has no wide
// path).  RIPTIDE_AMD_SNR_WIDE=0 drops the cap (A/B).
static bool wide_snr(const FfaXform& X, int smax, bool snr_epilogue, uint32_t max_width)
{
    if (!snr_epilogue || smax > 5 || smax == kPack2) return false;
    if (snr_group((int)X.p) != 16 || (int)max_width <= kSnrWin || max_width >= X.p) return false;
    if (const char* e = std::getenv("RIPTIDE_AMD_SNR_WIDE"))
        if (e[0] == '0') return false;
    return true;
}

// Final tiles of the segmented S/N (ffa_kernels.hip snr_segments): one block
// of kSnrSegRows rows; off with the kernel's feature bit
// (RIPTIDE_AMD_CONE_FLAGS without kConeSnrSeg, A/B).
static bool seg_snr(const FfaXform& X, int smax, bool snr_epilogue, uint32_t max_width)
{
    if (!snr_epilogue || (smax != 4 && smax != 5)) return false;
    if (!snr_seg_ok((int)X.p, (int)max_width, 1)) return false;
    if (const char* e = std::getenv("RIPTIDE_AMD_CONE_FLAGS"))
        if (!(std::strtoul(e, nullptr, 0) & kConeSnrSeg)) return false;
    return true;
}

static uint32_t final_tile_cap(const FfaXform& X, int smax, bool snr_epilogue, uint32_t max_width)
{
    if (seg_snr(X, smax, snr_epilogue, max_width)) return kSnrSegRows;
    if (!wide_snr(X, smax, snr_epilogue, max_width)) return 0;
    const int q = snr_wide_stride((int)X.p, (int)max_width);
    const int k = kLdsDataFloats / q;
    return k >= 8 ? (uint32_t)k : 0;
}

void build_exec_plan(const std::vector<FfaXform>& xforms, bool snr_epilogue, uint32_t num_widths,
                     uint64_t scratch_budget, ExecPlan& out, uint32_t max_width, uint32_t banks)
{
    if (banks != 1 && banks != 2) throw std::invalid_argument("scratch banks: 1 or 2");
    out = ExecPlan();
    out.xf = xforms;
    for (const FfaXform& X : xforms) {
        if (!merge_slots(X.p)) throw std::invalid_argument("phase bins too large for the LDS cone kernel");
        if ((uint64_t)X.m * X.p * 4u >= kMaxBlockBytes)
            throw std::invalid_argument("FFA transform block of " + std::to_string(X.m) + " x " + std::to_string(X.p) +
                                        " floats exceeds the 2 GiB range of the cone kernel");
    }
    const size_t nx = xforms.size();
    std::vector<uint32_t> xgroup(nx, 0);
    size_t g0 = 0;
    uint32_t group = 0;
    std::vector<std::vector<PassItems>> sched;
    while (g0 < nx) {
        // group [g0, g1): scratch fits the budget (always at least one transform)
        uint64_t scratch = 0;
        size_t g1 = g0;
        while (g1 < nx) {
            const uint64_t cells = ((uint64_t)xforms[g1].m * xforms[g1].p + 3) & ~(uint64_t)3;
            if (g1 > g0 && scratch + cells > scratch_budget) break;
            out.xf[g1].buf_off = scratch;
            xgroup[g1] = group;
            scratch += cells;
            ++g1;
        }
        out.scratch_floats = std::max(out.scratch_floats, scratch);
        sched.assign(g1 - g0, {});
        uint32_t gpasses = 0;
        for (size_t i = g0; i < g1; ++i) {
            plan_transform(out.xf[i], (uint32_t)i, merge_slots(out.xf[i].p),
                           final_tile_cap(out.xf[i], merge_slots(out.xf[i].p), snr_epilogue, max_width), sched[i - g0]);
            gpasses = std::max<uint32_t>(gpasses, (uint32_t)sched[i - g0].size());
        }
        out.max_passes = std::max(out.max_passes, gpasses);
        const size_t first_launch = out.launches.size();
        // one launch per (pass, kernel variant): a variant runs rows of exactly
        // its slot width (buckets <= 5), so no lane-slot is wasted
        std::vector<int> buckets;
        for (size_t i = g0; i < g1; ++i) buckets.push_back(merge_slots(out.xf[i].p));
        std::sort(buckets.begin(), buckets.end());
        buckets.erase(std::unique(buckets.begin(), buckets.end()), buckets.end());
        for (uint32_t k = 0; k < gpasses; ++k) {
            // merge-only and final (fused S/N) units in separate launches, so
            // each runs a kernel instance without the other's code
            for (const int bucket : buckets) for (int fin = 0; fin < 2; ++fin) {
                Launch L;
                L.snr = (uint32_t)fin;
                L.smax = (uint32_t)bucket;
                L.first = (uint32_t)out.items.size();
                L.group = group;
                L.pass = k;
                for (size_t i = g0; i < g1; ++i) {
                    auto& sp = sched[i - g0];
                    const uint32_t P = (uint32_t)sp.size();
                    if (k >= P || merge_slots(out.xf[i].p) != bucket) continue;
                    const FfaXform& X = out.xf[i];
                    const uint8_t src = k == 0 ? kSelLeaves : (((P - k) % 2 == 0) ? kSelPing : kSelPong);
                    const bool last = (k == P - 1);
                    if ((last && snr_epilogue) != (fin == 1)) continue;
                    const uint8_t dst = last ? (snr_epilogue ? kSelSnr : kSelPing)
                                             : (((P - 1 - k) % 2 == 0) ? kSelPing : kSelPong);
                    for (ConeItem it : sp[k].items) {
                        it.src = src;
                        it.dst = dst;
                        out.items.push_back(it);
                    }
                    const double cells = (double)X.m * X.p;
                    if (last && wide_snr(X, bucket, snr_epilogue, max_width)) L.wide_snr = 1;
                    L.cells += (uint64_t)X.m * X.p;
                    L.alg_bytes += 4.0 * cells + ((last && snr_epilogue) ? 4.0 * X.rows_eval * num_widths : 4.0 * cells);
                    L.moved_bytes += sp[k].read + ((last && snr_epilogue) ? 4.0 * X.rows_eval * num_widths : sp[k].written);
                }
                L.count = (uint32_t)out.items.size() - L.first;
                // longest first, so the launch tail is made of the cheapest units
                std::stable_sort(out.items.begin() + L.first, out.items.end(),
                                 [&](const ConeItem& x, const ConeItem& y) {
                                     return item_cost(x, out.xf[x.xform]) > item_cost(y, out.xf[y.xform]);
                                 });
                if (!L.count) continue;
                // whole-node units of every size in one launch, longest first
                // (one launch per register-row class, as before round 4, left
                // CUs idle at each class's drain: cfg2 7.22 -> 7.10, cfg3
                // 1.864 -> 1.809, cfg1 0.285 -> 0.263 ms per trial, same S/N)
                out.launches.push_back(L);
            }
        }
        // within the group: every merge-only launch first (in pass order),
        // then the final ones -- a final launch of pass k reads only the
        // merge-only pass k - 1 output of its own transform, so the order is
        // valid, and a second group can run its merge-only launches while
        // this group runs its finals (co-scheduling)
        std::stable_partition(out.launches.begin() + first_launch, out.launches.end(),
                              [](const Launch& L) { return L.snr == 0; });
        g0 = g1;
        ++group;
    }
    out.groups = group;
    out.bank_floats = out.scratch_floats;
    out.banks = group > 1 ? banks : 1;
    if (out.banks == 2) {
        for (size_t i = 0; i < nx; ++i)
            if (xgroup[i] & 1u) out.xf[i].buf_off += out.bank_floats;
        out.scratch_floats = 2 * out.bank_floats;
    }
    // host-built metadata of the tile items (trial-independent, shared by a
    // launch's whole batch)
    std::vector<int> slot_rw(out.items.size(), 0);
    std::vector<bool> packed(out.items.size(), false);
    std::vector<int> smax_of(out.items.size(), 0);
    for (const Launch& L : out.launches) {
        // row-slot tables for the kernel instances that use them (SMAX <= 5)
        const int rw = L.smax <= 5 ? (L.rw ? (int)L.rw : merge_rows_per_wave((int)L.smax)) : 0;
        for (uint32_t i = L.first; i < L.first + L.count; ++i) {
            slot_rw[i] = rw;
            packed[i] = L.smax == (uint32_t)kPack2;
            smax_of[i] = (int)L.smax;
        }
    }
    for (size_t i = 0; i < out.items.size(); ++i) {
        ConeItem& it = out.items[i];
        it.pad = kNoBlob;
        // whole units: a descriptor table only when it fits the LDS area
        // (otherwise the kernel derives the node partition on the fly);
        // kPack2 units always have one (in their level buffer)
        if (!packed[i] && it.mode != kModeTile &&
            ((uint64_t)it.levels * it.node_size > (uint64_t)kDescEntries || it.node_size > (uint32_t)kMaxRows))
            continue;
        it.pad = (uint32_t)out.blob.size();
        build_tile_blob(it, out.xf[it.xform].p, slot_rw[i], smax_of[i], out.blob);
    }
    validate_exec_plan(out, snr_epilogue);
}

// Row slots of one merge step (output level with n rows, descriptors d):
// rows in order, a pair where rows r, r + 1 share head and tail rows with
// shifts s, s + 1 (never carried rows), else a half where
// they share only the head row (neither carried), filled into the slots
// g = wave + 8q of the wave's register rows 2q, 2q + 1 (capacity 2, or 1 for
// the last slot of an odd RW).  Every slot is filled to its capacity (a pair
// or half split into two rows where needed), so n <= 8 RW rows always fit.
static void build_row_slots(const uint32_t* d, uint32_t n, uint32_t p, int rw, std::vector<uint32_t>& slots)
{
    struct Item { uint32_t r; uint32_t kind; };   // kSlotOne (a single row), kSlotPair or kSlotHalf
    std::vector<Item> items;
    for (uint32_t r = 0; r < n;) {
        const uint32_t a = d[r];
        const bool carried = ((a >> 10) & 1023u) == kCarriedRow;
        if (r + 1 < n && ((a ^ d[r + 1]) & 0xFFFFFu) == 0 && !carried && (d[r + 1] >> 20) == ((a >> 20) + 1) % p) {
            items.push_back({r, kSlotPair});
            r += 2;
        } else if (r + 1 < n && ((a ^ d[r + 1]) & 1023u) == 0 && !carried &&
                   ((d[r + 1] >> 10) & 1023u) != kCarriedRow) {
            items.push_back({r, kSlotHalf});
            r += 2;
        } else {
            items.push_back({r, kSlotOne});
            r += 1;
        }
    }
    const int Q = (rw + 1) / 2;
    slots.clear();
    size_t c = 0;
    for (int g = 0; c < items.size(); ++g) {
        if (g >= kConeWaves * Q) throw std::runtime_error("schedule: merge level exceeds the register rows");
        const int cap = (g / kConeWaves == Q - 1 && (rw & 1)) ? 1 : 2;
        Item& A = items[c];
        if (A.kind != kSlotOne && cap == 2) {
            slots.push_back(A.r | ((A.r + 1) << 10) | (A.kind << 20));
            ++c;
            continue;
        }
        const uint32_t ra = A.r;
        if (A.kind != kSlotOne) {   // split: row A alone, its partner stays next
            A.r += 1;
            A.kind = kSlotOne;
        } else {
            ++c;
        }
        if (cap == 1 || c == items.size()) {
            slots.push_back(ra | (kSlotOne << 20));
            continue;
        }
        Item& B = items[c];
        const uint32_t rb = B.r;
        if (B.kind != kSlotOne) {
            B.r += 1;
            B.kind = kSlotOne;
        } else {
            ++c;
        }
        slots.push_back(ra | (rb << 10) | (kSlotTwo << 20));
    }
}

void build_tile_blob(const ConeItem& it, uint32_t p, int slot_rw, int smax, std::vector<uint32_t>& out)
{
    const bool packed = smax == kPack2;
    const bool resolved = slot_rw > 0 && resolved_slots(smax);
    struct R { uint32_t size, lo, hi; uint32_t start; uint32_t base; };
    const int L = it.levels;
    const bool tile = it.mode == kModeTile;
    // level l: the row ranges of the unit (tile: 2^l ranges of the dependency
    // cone, children of range j at 2j (head) and 2j + 1 (tail) -- the planner
    // guarantees every node above the bottom has >= 2 rows; whole unit: the
    // node, one range per level)
    std::vector<std::vector<R>> lv(L + 1);
    lv[0].push_back({it.node_size, it.s0, it.s1 - 1, it.node_start, 0});
    for (int l = 1; l <= L; ++l) {
        if (!tile) {
            lv[l].push_back(lv[0][0]);
            continue;
        }
        for (const R& r : lv[l - 1]) {
            const uint32_t sh = r.size >> 1, st = r.size - sh;
            const float kh = merge_coef(sh, r.size), kt = merge_coef(st, r.size);
            lv[l].push_back({sh, merge_index(kh, r.lo), merge_index(kh, r.hi), r.start, 0});
            lv[l].push_back({st, merge_index(kt, r.lo), merge_index(kt, r.hi), r.start + sh, 0});
        }
    }
    uint32_t nrows[kMaxLevels + 1] = {}, doff[kMaxLevels + 1] = {};
    uint32_t entries = 0;
    for (int l = 0; l <= L; ++l) {
        uint32_t b = 0;
        for (R& r : lv[l]) {
            r.base = b;
            b += r.hi - r.lo + 1;
        }
        nrows[l] = b;
        doff[l] = entries;
        if (l < L) entries += b;
    }
    const size_t o = out.size();
    const uint32_t nruns = (uint32_t)lv[L].size(), nb = nrows[L];
    // [header | descriptors | bottom-row offsets | row slots] goes to LDS;
    // the DMA runs behind them are read by the kernel's scalar loads only.
    // The descriptor table is filled first, the slot tables after it.
    std::vector<uint32_t> desc_v(entries);
    uint32_t* desc = desc_v.data();
    for (int l = 0; l < L; ++l) {
        if (!tile) {
            // whole unit (cone_kernel row_desc): row r of depth l lies in the
            // depth-l node of the rows >> 1 split tree; size-1 nodes are carried
            for (uint32_t r = 0; r < nrows[l]; ++r) {
                uint32_t a0 = 0, sz = it.node_size;
                for (int d = 0; d < l; ++d)
                    if (sz > 1) {
                        const uint32_t hs = sz >> 1;
                        if (r - a0 < hs) sz = hs;
                        else {
                            a0 += hs;
                            sz -= hs;
                        }
                    }
                uint32_t word;
                if (sz <= 1) {
                    word = r | (kCarriedRow << 10);
                } else {
                    const uint32_t s = r - a0, hs = sz >> 1, ts = sz - hs;
                    const uint32_t hh = merge_index(merge_coef(hs, sz), s);
                    const uint32_t tt = merge_index(merge_coef(ts, sz), s);
                    word = (a0 + hh) | ((a0 + hs + tt) << 10) | (((s - tt) % p) << 20);
                }
                desc[doff[l] + r] = word;
            }
            continue;
        }
        // tile unit: output row r of level l within range j of its level
        size_t j = 0;
        for (uint32_t r = 0; r < nrows[l]; ++r) {
            while (j + 1 < lv[l].size() && lv[l][j + 1].base <= r) ++j;
            const R& g = lv[l][j];
            const uint32_t u = g.lo + (r - g.base);
            const R& H = lv[l + 1][2 * j];
            const R& T = lv[l + 1][2 * j + 1];
            const uint32_t hs = g.size >> 1, ts = g.size - hs;
            const uint32_t hh = merge_index(merge_coef(hs, g.size), u);
            const uint32_t tt = merge_index(merge_coef(ts, g.size), u);
            const uint32_t h = H.base + hh - H.lo, t = T.base + tt - T.lo;
            const uint32_t sh = (u - tt) % p;
            desc[doff[l] + r] = h | (t << 10) | (sh << 20);
        }
    }
    // bottom level: one DMA run per range, each at its own 16-byte phase,
    // consecutive in LDS; issued as segments of <= 64 16-byte chunks (one
    // LDS-DMA wave instruction each: LDS chunk c0, chunks n, source chunk g)
    std::vector<uint32_t> loff_v(nb), segs;
    uint32_t cb = 0;
    for (uint32_t ri = 0; ri < nruns; ++ri) {
        const R& g = lv[L][ri];
        const uint32_t first = (g.start + g.lo) * p;
        const uint32_t al = first & 3u, cnt = g.hi - g.lo + 1;
        const uint32_t nch = (cnt * p + al + 3) >> 2;
        for (uint32_t r = 0; r < cnt; ++r) loff_v[g.base + r] = 4 * cb + al + r * p;
        for (uint32_t c = 0; c < nch; c += 64) {
            segs.push_back(cb + c);
            segs.push_back(std::min<uint32_t>(64u, nch - c));
            segs.push_back((first - al) / 4 + c);
            segs.push_back(0u);
        }
        cb += nch;
    }
    // row slots of every merge step (the kernel's step order: two levels per
    // step where no level below the output holds size-1 nodes)
    std::vector<uint32_t> slot_area;
    uint32_t slot_off[kMaxLevels + 1] = {};
    uint32_t zero_row = 0;
    if (packed) {
        // kPack2: every lane resolves its own row, so a two-level step gets
        // its rows pre-resolved (one 8-byte read per row instead of three
        // dependent descriptor reads): the four source rows of level lo + 2
        // and the three rolls (sH, sh, (sh + sT) mod p), and only the levels
        // single steps read keep their descriptors
        std::vector<bool> keep(L + 1, false), fused(L + 1, false);
        std::vector<uint32_t> rel(L + 1, 0);
        for (int l = L - 1; l >= 0;) {
            const bool two = l >= 1 && (tile || (it.node_size >> l) >= 2);
            const int lo = two ? l - 1 : l;
            if (!two) {
                keep[lo] = true;
            } else {
                fused[lo] = true;
                rel[lo] = (uint32_t)slot_area.size();   // even: two words per row
                for (uint32_t r = 0; r < nrows[lo]; ++r) {
                    const uint32_t d0 = desc[doff[lo] + r];
                    const uint32_t dh = desc[doff[lo + 1] + (d0 & 1023u)];
                    const uint32_t dt = desc[doff[lo + 1] + ((d0 >> 10) & 1023u)];
                    const uint32_t sh = d0 >> 20, sH = dh >> 20, sTT = ((d0 >> 20) + (dt >> 20)) % p;
                    slot_area.push_back((dh & 1023u) | (((dh >> 10) & 1023u) << 10) | ((dt & 1023u) << 20));
                    slot_area.push_back(((dt >> 10) & 1023u) | (sH << 10) | (sh << 16) | (sTT << 22));
                }
            }
            l = lo - 1;
        }
        // compact descriptor table: the kept levels only
        std::vector<uint32_t> dc;
        for (int l = 0; l < L; ++l) {
            const uint32_t o0 = doff[l];
            doff[l] = (uint32_t)dc.size();
            if (keep[l]) dc.insert(dc.end(), desc_v.begin() + o0, desc_v.begin() + o0 + nrows[l]);
        }
        desc_v.swap(dc);
        desc = desc_v.data();
        entries = (uint32_t)desc_v.size();
        // the step tables start 8-byte aligned (uint2 reads)
        const uint32_t base0 = kBlobHeader + entries + nb;
        if (base0 & 1u) slot_area.insert(slot_area.begin(), 0u);
        const uint32_t base = base0 + (base0 & 1u);
        for (int l = 0; l <= L; ++l)
            if (fused[l]) slot_off[l] = base + rel[l];
    } else if (resolved) {
        // whole units with an even number of levels fuse every step: the
        // deepest step's carried (size-1) middle-level nodes read their
        // missing operand from a -0.0 row past the fill (kHdrZero)
        if (!tile && L >= 2 && (L % 2) == 0 && 4 * cb + 64 * (uint32_t)smax <= (uint32_t)kLdsDataFloats) zero_row = 4 * cb;
        // 4/5-slot variants: every step's row slots with their rows resolved
        // (resolved_slots): a lane reads its slot's row A (lanes 0-31) or row
        // B (32-63) as one 16-byte entry -- LDS offsets of the source rows
        // (the first step's in the fill layout), the rolls and the slot word
        // -- instead of a chain of descriptor reads; the descriptor table is
        // not stored.
        std::vector<uint32_t> sl;
        const uint32_t base0 = kBlobHeader + nb;
        const uint32_t base = (base0 + 3u) & ~3u;       // 16-byte aligned tables
        slot_area.assign(base - base0, 0u);
        for (int l = L - 1; l >= 0;) {
            const bool two = l >= 1 && (tile || zero_row || (it.node_size >> l) >= 2);
            const int lo = two ? l - 1 : l;
            const bool first = l == L - 1;
            build_row_slots(desc + doff[lo], nrows[lo], p, slot_rw, sl);
            slot_off[lo] = (uint32_t)(base0 + slot_area.size());
            slot_area.insert(slot_area.end(), {(uint32_t)sl.size(), 0u, 0u, 0u});
            auto off = [&](uint32_t row) { return first ? loff_v[row] : row * p; };
            auto entry = [&](uint32_t r, uint32_t* e) {
                const uint32_t d0 = desc[doff[lo] + r];
                if (two) {
                    const uint32_t dh = desc[doff[lo + 1] + (d0 & 1023u)];
                    const uint32_t dt = desc[doff[lo + 1] + ((d0 >> 10) & 1023u)];
                    // a carried middle-level node: its row is the level-below
                    // row plus the -0.0 row (zero_row; only the deepest step)
                    const bool ch = ((dh >> 10) & 1023u) == kCarriedRow, ct = ((dt >> 10) & 1023u) == kCarriedRow;
                    if ((ch || ct) && !(zero_row && first))
                        throw std::runtime_error("schedule: fused step over carried nodes without a zero row");
                    const uint32_t sh = d0 >> 20, sH = ch ? 0u : dh >> 20;
                    const uint32_t sTT = ((d0 >> 20) + (ct ? 0u : dt >> 20)) % p;
                    e[0] = off(dh & 1023u) | ((ch ? zero_row : off((dh >> 10) & 1023u)) << 16);
                    e[1] = off(dt & 1023u) | ((ct ? zero_row : off((dt >> 10) & 1023u)) << 16);
                    e[2] = sH | (sh << 10) | (sTT << 20);
                } else {
                    const uint32_t tc = (d0 >> 10) & 1023u, car = tc == kCarriedRow;
                    const uint32_t oh = off(d0 & 1023u);
                    e[0] = oh | ((car ? oh : off(tc)) << 16);
                    e[1] = 0u;
                    e[2] = (d0 >> 20) | (car << 30);
                }
            };
            // wave-major halves: row A entries of wave w's slots q at
            // [w Q + q], row B entries at [8 Q + w Q + q] (16 bytes each), so
            // the 32 lanes of a half read consecutive entries (no bank
            // conflicts; slot g = w + 8 q is the wave's q-th slot)
            const int Q = (slot_rw + 1) / 2;
            const size_t t0 = slot_area.size();
            slot_area.resize(t0 + 4 * 2 * (size_t)kConeWaves * Q, 0u);
            for (size_t g = 0; g < sl.size(); ++g) {
                const uint32_t sw = sl[g];
                const size_t wq = (g % kConeWaves) * Q + g / kConeWaves;
                uint32_t* ea = slot_area.data() + t0 + 4 * wq;
                uint32_t* eb = slot_area.data() + t0 + 4 * ((size_t)kConeWaves * Q + wq);
                entry(sw & 1023u, ea);
                ea[3] = sw;
                if ((sw >> 20) == kSlotTwo || (sw >> 20) == kSlotHalf) entry((sw >> 10) & 1023u, eb);
            }
            l = lo - 1;
        }
        if (slot_area.size() > (size_t)(kAuxMetaWords - kBlobHeader - nb))
            throw std::runtime_error("schedule: resolved row-slot tables exceed their LDS area");
        entries = 0;   // no descriptor table in LDS
        for (int l = 0; l <= L; ++l) doff[l] = 0;
    } else if (slot_rw > 0) {
        std::vector<uint32_t> sl;
        for (int l = L - 1; l >= 0;) {
            const bool two = l >= 1 && (tile || (it.node_size >> l) >= 2);
            const int lo = two ? l - 1 : l;
            build_row_slots(desc + doff[lo], nrows[lo], p, slot_rw, sl);
            slot_off[lo] = (uint32_t)(kBlobHeader + entries + nb + slot_area.size());
            slot_area.push_back((uint32_t)sl.size());
            slot_area.insert(slot_area.end(), sl.begin(), sl.end());
            l = lo - 1;
        }
        if (slot_area.size() > (size_t)kSlotWords) throw std::runtime_error("schedule: row-slot tables exceed their LDS area");
    }
    const uint32_t nsegs = (uint32_t)(segs.size() / 4);
    {
        // wave-major order: segment g (issued by wave g % 8) at
        // (g % 8) * K + g / 8, K = ceil(nsegs / 8), so a wave's lanes load
        // its segments from consecutive 16-byte entries
        const uint32_t K = (nsegs + kConeWaves - 1) / kConeWaves;
        std::vector<uint32_t> wm((size_t)4 * K * kConeWaves, 0u);
        for (uint32_t g = 0; g < nsegs; ++g)
            std::copy(segs.begin() + 4 * g, segs.begin() + 4 * g + 4, wm.begin() + 4 * ((g % kConeWaves) * K + g / kConeWaves));
        segs.swap(wm);
    }
    if (nsegs > (uint32_t)(kConeWaves * 64)) throw std::runtime_error("schedule: unit fill exceeds the DMA segment table");
    const size_t lds_words = kBlobHeader + entries + nb + slot_area.size();
    const size_t runoff = (lds_words + 3) & ~(size_t)3;
    const size_t words = runoff + segs.size();
    out.resize(o + ((words + 3) & ~(size_t)3), 0u);
    uint32_t* w = out.data() + o;
    for (int l = 0; l <= L; ++l) {
        w[kHdrRows + l] = nrows[l];
        w[kHdrDesc + l] = doff[l];
        w[kHdrSlotOff + l] = slot_off[l];
    }
    w[kHdrRuns] = nsegs;
    w[kHdrEntries] = entries;
    w[kHdrBottom] = nb;
    w[kHdrSlotWords] = (uint32_t)slot_area.size();
    w[kHdrRunOff] = (uint32_t)runoff;
    w[kHdrFill] = cb;
    w[kHdrZero] = zero_row;
    if (entries) std::copy(desc_v.begin(), desc_v.begin() + entries, w + kBlobHeader);
    std::copy(loff_v.begin(), loff_v.end(), w + kBlobHeader + entries);
    std::copy(slot_area.begin(), slot_area.end(), w + kBlobHeader + entries + nb);
    std::copy(segs.begin(), segs.end(), w + runoff);
}

// The 4-slot roll table sits at kLut4Off, past every 4-slot unit's blob LDS
// part.  Worst case of that part: the header, <= 72 bottom-row offsets (the
// 4-slot capacity: 8 waves x kRw4 register rows), 16-byte alignment, and the
// resolved slot tables of <= 4 merge steps (whole units have <= 7 levels, of
// which only the deepest can hold size-1 nodes: 1 + ceil(6 / 2) steps; tiles
// <= kMaxTileLevels = 6 fused levels: 3 steps), each 4 header words + two
// 16-byte entries per slot of every wave.  So a tile never needs to shrink
// for the table, and validate_blob's check below can only fire on a broken
// build.
constexpr int kMaxSteps4 = 4;
constexpr int kBlobLds4Worst =
    kBlobHeader + kConeWaves * kRw4 + 3 + kMaxSteps4 * (4 + 4 * 2 * kConeWaves * ((kRw4 + 1) / 2));
static_assert(kBlobLds4Worst <= kLut4Off, "4-slot unit blobs may overlap the roll table");
static_assert((kMaxTileLevels + 1) / 2 <= kMaxSteps4, "tile steps");

// A unit's blob as the kernel will read it: the DMA segments tile the fill
// [0, fill chunks) in order, each <= 64 chunks inside the level buffer; every
// row-slot table covers its step's output rows exactly once, a pair's rows
// sharing head and tail rows with consecutive shifts (never carried rows),
// within the register rows of the launch's kernel instance.
static void validate_blob(const ConeItem& it, uint32_t p, int smax, int rw, const uint32_t* w)
{
    const uint32_t L = it.levels;
    const uint32_t nseg = w[kHdrRuns], entries = w[kHdrEntries], nb = w[kHdrBottom];
    const uint32_t slot_words = w[kHdrSlotWords], runoff = w[kHdrRunOff], fill = w[kHdrFill];
    if (runoff < (uint32_t)kBlobHeader + entries + nb + slot_words || (runoff & 3u) || nb != w[kHdrRows + L])
        throw std::runtime_error("schedule: malformed unit blob header");
    if (4 * fill > (uint32_t)kLdsBufFloats) throw std::runtime_error("schedule: unit fill exceeds the LDS level buffer");
    // a 4-slot row-slot unit's roll table follows its blob's LDS part
    if (smax == 4 && slot_words && runoff > (uint32_t)kLut4Off)
        throw std::runtime_error("schedule: unit blob overlaps the roll table");
    uint32_t c = 0;
    const uint32_t K = (nseg + kConeWaves - 1) / kConeWaves;   // wave-major segment order
    for (uint32_t i = 0; i < nseg; ++i) {
        const uint32_t* g = w + runoff + 4 * ((i % kConeWaves) * K + i / kConeWaves);
        if (g[0] != c || g[1] == 0 || g[1] > 64) throw std::runtime_error("schedule: DMA segments do not tile the fill");
        c += g[1];
    }
    if (c != fill) throw std::runtime_error("schedule: DMA segments do not tile the fill");
    const uint32_t* desc = w + kBlobHeader;
    if (smax != kPack2 && !(resolved_slots(smax) && slot_words))
        for (uint32_t l = 0; l < L; ++l)
            if (w[kHdrDesc + l] + w[kHdrRows + l] > entries) throw std::runtime_error("schedule: descriptor table overrun");
    const bool tile = it.mode == kModeTile;
    if (smax == kPack2) {
        // pre-resolved two-level steps: source rows inside level lo + 2, rolls < p
        for (int l = (int)L - 1; l >= 0;) {
            const bool two = l >= 1 && (tile || (it.node_size >> l) >= 2);
            const int lo = two ? l - 1 : l;
            if (two) {
                const uint32_t so = w[kHdrSlotOff + lo], n = w[kHdrRows + lo], nsrc = w[kHdrRows + lo + 2];
                if (!so || (so & 1u) || so + 2 * n > runoff) throw std::runtime_error("schedule: step table outside the blob");
                for (uint32_t r = 0; r < n; ++r) {
                    const uint32_t a = w[so + 2 * r], b = w[so + 2 * r + 1];
                    const uint32_t s1 = (b >> 10) & 63u, s2 = (b >> 16) & 63u, s3 = (b >> 22) & 63u;
                    if ((a & 1023u) >= nsrc || ((a >> 10) & 1023u) >= nsrc || ((a >> 20) & 1023u) >= nsrc ||
                        (b & 1023u) >= nsrc || s1 >= p || s2 >= p || s3 >= p)
                        throw std::runtime_error("schedule: bad step table entry");
                }
            } else if (w[kHdrDesc + lo] + w[kHdrRows + lo] > entries) {
                throw std::runtime_error("schedule: descriptor table overrun");
            }
            l = lo - 1;
        }
        return;
    }
    if (!slot_words) {
        if (smax <= 5 && L > 0) throw std::runtime_error("schedule: unit without row-slot tables");
        return;
    }
    if (resolved_slots(smax)) {
        const int Q = (rw + 1) / 2;
        // The zero row lies past the fill; a final whole unit's output level
        // (S/N stride) or the segmented S/N's maxima / exchange areas may
        // cover it.  That is allowed: the kernel writes it at the workgroup's
        // start and again after every trial's S/N (behind the trial loop's
        // barrier, ffa_kernels.hip cone_kernel), before the next trial's
        // first merge step reads it; the next trial's DMA (below 4 * fill)
        // never touches it.
        const uint32_t zero_row = w[kHdrZero];
        if (zero_row && (tile || (L % 2) || zero_row < 4 * fill || zero_row + 64 * (uint32_t)smax > (uint32_t)kLdsDataFloats))
            throw std::runtime_error("schedule: bad zero row");
        for (int l = (int)L - 1; l >= 0;) {
            const bool two = l >= 1 && (tile || zero_row || (it.node_size >> l) >= 2);
            const int lo = two ? l - 1 : l;
            const uint32_t n = w[kHdrRows + lo], so = w[kHdrSlotOff + lo];
            if ((so & 3u) || so < (uint32_t)kBlobHeader + nb || so + 4 > runoff)
                throw std::runtime_error("schedule: row-slot table outside the blob");
            const uint32_t ns = w[so];
            if (ns > (uint32_t)(kConeWaves * Q) || so + 4 + 8 * (uint32_t)(kConeWaves * Q) > runoff)
                throw std::runtime_error("schedule: row-slot table overrun");
            std::vector<uint8_t> seen(n, 0);
            auto check_entry = [&](const uint32_t* e) {
                const uint32_t s1 = e[2] & 1023u, s2 = (e[2] >> 10) & 1023u, s3 = (e[2] >> 20) & 1023u;
                const uint32_t top = (uint32_t)kLdsBufFloats;
                if (s1 >= p || (two && (s2 >= p || s3 >= p)) || (e[0] & 0xFFFFu) + p > top ||
                    (e[0] >> 16) + p > top || (two && ((e[1] & 0xFFFFu) + p > top || (e[1] >> 16) + p > top)))
                    throw std::runtime_error("schedule: bad resolved row entry");
            };
            for (uint32_t g = 0; g < ns; ++g) {
                const uint32_t wq = (g % kConeWaves) * (uint32_t)Q + g / kConeWaves;
                const uint32_t* e = w + so + 4 + 4 * wq;
                const uint32_t* eb = w + so + 4 + 4 * ((uint32_t)(kConeWaves * Q) + wq);
                const uint32_t sw = e[3], ra = sw & 1023u, rb = (sw >> 10) & 1023u, kind = sw >> 20;
                const int q = (int)g / kConeWaves;
                const bool two_rows = kind != kSlotOne;
                if (kind > kSlotHalf || ra >= n || (two_rows && (rb >= n || 2 * q + 1 >= rw)) ||
                    ((kind == kSlotPair || kind == kSlotHalf) && rb != ra + 1))
                    throw std::runtime_error("schedule: bad row slot");
                if (seen[ra]++ || (two_rows && seen[rb]++)) throw std::runtime_error("schedule: row slot covers a row twice");
                check_entry(e);
                if (kind == kSlotTwo || kind == kSlotHalf) check_entry(eb);
                // a half's rows share the head term: the same head source
                // offsets (and, two levels, the same head-tail roll), not carried
                if (kind == kSlotHalf &&
                    ((two ? (e[0] != eb[0] || (e[2] & 1023u) != (eb[2] & 1023u))
                          : ((e[0] & 0xFFFFu) != (eb[0] & 0xFFFFu))) ||
                     (!two && (((e[2] >> 30) & 1u) || ((eb[2] >> 30) & 1u)))))
                    throw std::runtime_error("schedule: row half without a shared head term");
            }
            for (uint32_t r = 0; r < n; ++r)
                if (!seen[r]) throw std::runtime_error("schedule: row-slot table misses a row");
            l = lo - 1;
        }
        return;
    }
    const int Q = (rw + 1) / 2;
    for (int l = (int)L - 1; l >= 0;) {
        const bool two = l >= 1 && (tile || (it.node_size >> l) >= 2);
        const int lo = two ? l - 1 : l;
        const uint32_t n = w[kHdrRows + lo], so = w[kHdrSlotOff + lo];
        if (so < (uint32_t)kBlobHeader + entries + nb || so >= runoff) throw std::runtime_error("schedule: row-slot table outside the blob");
        const uint32_t ns = w[so];
        if (ns > (uint32_t)(kConeWaves * Q) || so + 1 + ns > runoff) throw std::runtime_error("schedule: row-slot table overrun");
        std::vector<uint8_t> seen(n, 0);
        const uint32_t* d = desc + w[kHdrDesc + lo];
        for (uint32_t g = 0; g < ns; ++g) {
            const uint32_t sw = w[so + 1 + g], ra = sw & 1023u, rb = (sw >> 10) & 1023u, kind = sw >> 20;
            const int q = (int)g / kConeWaves;
            const bool two_rows = kind != kSlotOne;
            if (kind > kSlotHalf || ra >= n || (two_rows && (rb >= n || 2 * q + 1 >= rw)))
                throw std::runtime_error("schedule: bad row slot");
            if (seen[ra]++ || (two_rows && seen[rb]++)) throw std::runtime_error("schedule: row slot covers a row twice");
            if (kind == kSlotHalf) {
                const uint32_t a = d[ra], b = d[rb];
                if (rb != ra + 1 || ((a ^ b) & 1023u) || ((a >> 10) & 1023u) == kCarriedRow ||
                    ((b >> 10) & 1023u) == kCarriedRow)
                    throw std::runtime_error("schedule: row half without a shared head row");
            }
            if (kind == kSlotPair) {
                const uint32_t a = d[ra], b = d[rb];
                if (rb != ra + 1 || ((a ^ b) & 0xFFFFFu) || ((a >> 10) & 1023u) == kCarriedRow ||
                    (b >> 20) != ((a >> 20) + 1) % p)
                    throw std::runtime_error("schedule: row pair without shared head/tail rows");
            }
        }
        for (uint32_t r = 0; r < n; ++r)
            if (!seen[r]) throw std::runtime_error("schedule: row-slot table misses a row");
        l = lo - 1;
    }
}

void validate_exec_plan(const ExecPlan& ex, bool snr_epilogue)
{
    std::vector<uint64_t> covered(ex.xf.size(), 0);
    std::vector<uint32_t> last_pass(ex.xf.size(), 0);
    for (const Launch& L : ex.launches)
        for (uint32_t i = L.first; i < L.first + L.count; ++i)
            last_pass[ex.items[i].xform] = std::max(last_pass[ex.items[i].xform], L.pass);
    for (const FfaXform& X : ex.xf) {
        if ((uint64_t)X.m * X.p * 4u >= kMaxBlockBytes) throw std::runtime_error("schedule: transform block over 2 GiB");
        if (X.buf_off + (((uint64_t)X.m * X.p + 3) & ~(uint64_t)3) > ex.scratch_floats)
            throw std::runtime_error("schedule: transform scratch outside the ping/pong buffers");
    }
    for (const Launch& L : ex.launches) {
        if (L.first + L.count > ex.items.size()) throw std::runtime_error("schedule: launch outside the item list");
        for (uint32_t i = L.first; i < L.first + L.count; ++i) {
            const ConeItem& it = ex.items[i];
            if (it.xform >= ex.xf.size()) throw std::runtime_error("schedule: item of an unknown transform");
            const FfaXform& X = ex.xf[it.xform];
            if (merge_slots(X.p) != (int)L.smax) throw std::runtime_error("schedule: item in the wrong kernel variant");
            if (it.s1 <= it.s0 || it.s1 > it.node_size || (uint64_t)it.node_start + it.node_size > X.m)
                throw std::runtime_error("schedule: tile outside its node");
            int rows;
            if (it.mode == kModeTile) {
                const ConeNeed n = cone_need(it.node_size, it.s0, it.s1, it.levels, X.p);
                if (n.degenerate || n.max_rows > kMaxRows || n.max_floats > kLdsDataFloats || n.ranges > kMaxRanges ||
                    it.levels > kMaxTileLevels)
                    throw std::runtime_error("schedule: tile exceeds the LDS budget");
                rows = n.max_rows;
            } else {
                if ((int)it.node_size * (int)X.p > kLdsDataFloats || it.node_size > (uint32_t)kMaxRows ||
                    it.levels > kMaxLevels || (1u << it.levels) < it.node_size)
                    throw std::runtime_error("schedule: whole node exceeds the LDS budget");
                rows = (int)it.node_size;
            }
            const ConeNeed need = it.mode == kModeTile ? cone_need(it.node_size, it.s0, it.s1, it.levels, X.p)
                                                       : ConeNeed{};
            const int bottom = it.mode == kModeTile ? need.rows_bottom : (int)it.node_size;
            if (4 * fill_chunks_bound(bottom, (int)X.p, it.mode == kModeTile ? 1 << it.levels : 1) > kLdsBufFloats)
                throw std::runtime_error("schedule: unit fill exceeds the LDS level buffer");
            if (L.smax == (uint32_t)kPack2) {
                // blob at the end of the level buffer, clear of the fill and every level
                if (it.pad == kNoBlob) throw std::runtime_error("schedule: short-row unit without a descriptor table");
                const uint32_t* h = ex.blob.data() + it.pad;
                const int top = std::max<int>(4 * (int)h[kHdrFill], rows * pack_stride((int)X.p));
                if (top + (int)h[kHdrRunOff] > kLdsBufFloats)
                    throw std::runtime_error("schedule: short-row unit and its descriptor table exceed the level buffer");
            } else if (it.mode == kModeTile && (need.entries > kDescEntries || it.pad == kNoBlob)) {
                throw std::runtime_error("schedule: tile descriptor table exceeds its LDS area");
            }
            // the 4/5-slot instances run only row-slot steps (ffa_kernels.hip
            // merge_levels): every unit with a merge level has its slot tables
            if (resolved_slots((int)L.smax) && it.levels > 0 &&
                (it.pad == kNoBlob || ex.blob[it.pad + kHdrSlotWords] == 0))
                throw std::runtime_error("schedule: 4/5-slot unit without row-slot tables");
            // the launch's kernel instance is the unit's kind (final: fused S/N)
            if ((it.dst == kSelSnr) != (L.snr != 0)) throw std::runtime_error("schedule: unit in a launch of the other kind");
            if (L.wide_snr && !L.snr) throw std::runtime_error("schedule: wide S/N on a merge-only launch");
            // the launch's kernel instance stages enough register rows for every level
            const int rw = L.rw ? (int)L.rw : merge_rows_per_wave((int)L.smax);
            if (it.pad != kNoBlob) {
                if ((size_t)it.pad + kBlobHeader > ex.blob.size()) throw std::runtime_error("schedule: blob outside the plan");
                validate_blob(it, X.p, (int)L.smax, rw, ex.blob.data() + it.pad);
            }
            if (rows > kConeWaves * rw * row_pack((int)L.smax) || rows > lds_row_capacity(X.p, (int)L.smax))
                throw std::runtime_error("schedule: unit rows exceed its kernel instance's register rows");
            if (L.pass == last_pass[it.xform]) {
                if (it.node_start != 0 || (snr_epilogue ? it.dst != kSelSnr : it.dst == kSelSnr))
                    throw std::runtime_error("schedule: bad final pass");
                covered[it.xform] += it.s1 - it.s0;
            }
        }
    }
    for (size_t t = 0; t < ex.xf.size(); ++t)
        if (covered[t] != ex.xf[t].m) throw std::runtime_error("schedule: final pass does not cover the transform");
}

}  // namespace rt

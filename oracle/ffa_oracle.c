/*
 * ffa_oracle.c -- clean-room CPU restatement of riptide's FFA periodogram hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in riptide_amd/ links, loads or calls this
 * file; it is the checker that tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg compare the HIP path against.  Parity of this restatement is
 * pinned against the reference itself (oracle/_ref, built from
 * /root/reference/riptide/cpp by oracle/Makefile) through the golden vectors in
 * tests/golden/ (tests/test_oracle_golden.py).
 *
 * Built strict (-ffp-contract=off, no fast-math): every expression below is
 * evaluated exactly as written.  Where the reference's compiled code differs from
 * its source text (g++ -O3 -ffast-math -march=native, setup.py:18), the emitted
 * form is restated explicitly and cited.
 *
 * Citations are path:line relative to /root/reference.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* FFA merge index.  transforms.hpp:17-22:                                    */
/*   kh = (head_rows - 1.0f) / (m - 1.0f);  h = (size_t)(kh * s + 0.5f)       */
/* The reference build contracts kh*s + 0.5f into one FMA (-march=native has  */
/* FMA3 and GCC contracts by default); mode 1 restates that, mode 0 is the    */
/* unfused source text.  tests/test_oracle_golden.py pins which one matches.  */
/* ------------------------------------------------------------------------- */
static int g_index_fma = 1;

void oracle_set_index_fma(int on) { g_index_fma = on; }

static size_t merge_index(float k, size_t s)
{
    const float fs = (float)s;
    float v;
    if (g_index_fma)
        v = fmaf(k, fs, 0.5f);
    else
        v = k * fs + 0.5f;
    return (size_t)v;
}

/* One merge step (transforms.hpp:13-27 + kernels.hpp:19-25):
 *   out[s][j] = H[h][j] + T[t][(j + shift) mod p],  shift = h + (s - (h + t))
 * with the size_t (mod 2^64) arithmetic of the reference. */
static void merge_rows(const float* head, size_t mh, const float* tail, size_t mt,
                       float* out, size_t m, size_t p)
{
    const float kh = ((float)mh - 1.0f) / ((float)m - 1.0f);
    const float kt = ((float)mt - 1.0f) / ((float)m - 1.0f);
    for (size_t s = 0; s < m; ++s) {
        const size_t h = merge_index(kh, s);
        const size_t t = merge_index(kt, s);
        const size_t b = s - (h + t);
        const size_t shift = (h + b) % p;
        const float* hr = head + h * p;
        const float* tr = tail + t * p;
        float* o = out + s * p;
        for (size_t j = 0; j < p; ++j) {
            size_t jj = j + shift;
            if (jj >= p) jj -= p;
            o[j] = hr[j] + tr[jj];
        }
    }
}

/* Recursive transform with the reference's split: head = rows >> 1
 * (block.hpp:30), children land in `tmp`, merged into `out` (transforms.hpp:30-50).
 * A one-row block is a copy; the two-row case of transforms.hpp:35-45 is the
 * general merge of two one-row children (kh = kt = 0). */
static void ffa_rec(const float* in, float* tmp, float* out, size_t m, size_t p)
{
    if (m == 1) {
        memcpy(out, in, p * sizeof(float));
        return;
    }
    const size_t mh = m >> 1;
    const size_t mt = m - mh;
    ffa_rec(in, out, tmp, mh, p);
    ffa_rec(in + mh * p, out + mh * p, tmp + mh * p, mt, p);
    merge_rows(tmp, mh, tmp + mh * p, mt, out, m, p);
}

/* ffa2 (python_bindings.cpp:72-84).  Returns 0, or -1 on allocation failure. */
int oracle_ffa2(const float* in, size_t rows, size_t cols, float* out)
{
    if (rows == 0 || cols == 0)
        return 0;
    float* tmp = (float*)malloc(rows * cols * sizeof(float));
    if (!tmp)
        return -1;
    ffa_rec(in, tmp, out, rows, cols);
    free(tmp);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Downsampling (downsample.hpp:21-82)                                        */
/* ------------------------------------------------------------------------- */
size_t oracle_downsampled_size(size_t n, double f)
{
    return (size_t)floor((double)n / f);
}

double oracle_downsampled_variance(size_t n, double f)
{
    const double k = floor(f);
    const double r = f - k;
    const double x = (double)oracle_downsampled_size(n, f) * r;
    if (x > 1.0)
        return f - 1.0 / 3.0;
    return (k - 1.0) * (k - 1.0) + 2.0 / 3.0 * (x * x) - x + 1.0;
}

/* out[k] = wmin*x[imin] + sum(x[imin+1..imax-1]) + wmax*x[imax], summed in that
 * order in float32 (downsample.hpp:55-80).  Caller checks 1 < f <= n. */
void oracle_downsample(const float* x, size_t n, double f, float* out)
{
    const size_t nout = oracle_downsampled_size(n, f);
    for (size_t k = 0; k < nout; ++k) {
        const double start = (double)k * f;
        const double end = start + f;
        const size_t imin = (size_t)floor(start);
        double dmax = floor(end);
        if (dmax > (double)n - 1.0)
            dmax = (double)n - 1.0;
        const size_t imax = (size_t)dmax;
        const float wmin = (float)((double)(imin + 1) - start);
        const float wmax = (float)(end - (double)imax);
        float acc = wmin * x[imin];
        for (size_t i = imin + 1; i < imax; ++i)
            acc += x[i];
        acc += wmax * x[imax];
        out[k] = acc;
    }
}

/* ------------------------------------------------------------------------- */
/* Boxcar S/N (snr.hpp:37-65, kernels.hpp:50-101)                             */
/* ------------------------------------------------------------------------- */
void oracle_circular_prefix_sum(const float* x, size_t n, size_t nsum, float* out)
{
    double acc = 0.0;
    const size_t jmax = n < nsum ? n : nsum;
    for (size_t j = 0; j < jmax; ++j) {
        acc += (double)x[j];
        out[j] = (float)acc;
    }
    if (nsum <= n)
        return;
    const float total = (float)acc;
    for (size_t i = n; i < nsum; ++i) {
        const size_t q = i / n;
        out[i] = out[i - q * n] + (float)q * total;
    }
}

static void snr_row(const float* row, size_t p, const uint64_t* widths, size_t nw,
                    float stdnoise, float* cps, float* out)
{
    uint64_t wmax = 0;
    for (size_t i = 0; i < nw; ++i)
        if (widths[i] > wmax)
            wmax = widths[i];
    oracle_circular_prefix_sum(row, p, p + (size_t)wmax, cps);
    const float sum = cps[p - 1];
    for (size_t iw = 0; iw < nw; ++iw) {
        const size_t w = (size_t)widths[iw];
        const float h = sqrtf((float)(p - w) / (float)(p * w));
        const float b = (float)w / (float)(p - w) * h;
        float dmax = cps[w] - cps[0];
        for (size_t i = 1; i < p; ++i) {
            const float d = cps[i + w] - cps[i];
            if (d > dmax)
                dmax = d;
        }
        out[iw] = ((h + b) * dmax - b * sum) / stdnoise;
    }
}

/* snr2 over a rows x cols block.  Caller validated widths (0 < w < cols) and
 * stdnoise > 0 (snr.hpp:14-31).  Returns -1 on allocation failure. */
int oracle_snr2(const float* x, size_t rows, size_t cols, const uint64_t* widths,
                size_t nw, float stdnoise, float* out)
{
    uint64_t wmax = 0;
    for (size_t i = 0; i < nw; ++i)
        if (widths[i] > wmax)
            wmax = widths[i];
    float* cps = (float*)malloc((cols + (size_t)wmax + 1) * sizeof(float));
    if (!cps)
        return -1;
    for (size_t r = 0; r < rows; ++r)
        snr_row(x + r * cols, cols, widths, nw, stdnoise, cps, out + r * nw);
    free(cps);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Periodogram plan and grid (periodogram.hpp:54-201)                         */
/* ------------------------------------------------------------------------- */
static size_t ceilshift(size_t rows, size_t cols, double pmax)
{
    /* periodogram.hpp:56, in the order the reference build evaluates it */
    return (size_t)ceil((double)cols * ((double)rows - 1.0) * (1.0 - (double)cols / pmax));
}

/* 0 ok, 1..6 = which argument check failed (periodogram.hpp:25-40) */
int oracle_periodogram_check(size_t n, double tsamp, double pmin, double pmax,
                             size_t bmin, size_t bmax)
{
    (void)n;
    if (!(tsamp > 0)) return 1;
    if (!(pmin > 0)) return 2;
    if (!(pmax > pmin)) return 3;
    if (!(bmin > 1)) return 4;
    if (!(bmax >= bmin)) return 5;
    if (!(pmin >= tsamp * (double)bmin)) return 6;
    return 0;
}

typedef struct {
    size_t rung;
    double f, tau;
    size_t n, bins, rows, rows_eval;
    float stdnoise;
} oracle_step;

/* Iterate over the (rung, bins) steps of the plan; calls cb for each. */
typedef void (*step_cb)(const oracle_step*, void*);

static void plan_walk(size_t n, double tsamp, double pmin, double pmax, size_t bmin,
                      size_t bmax, step_cb cb, void* ctx)
{
    const double ds_ini = pmin / (tsamp * (double)bmin);
    const double ds_geo = ((double)bmax + 1.0) / (double)bmin;
    const size_t nds = (size_t)ceil(log(pmax / pmin) / log(ds_geo));
    for (size_t ids = 0; ids < nds; ++ids) {
        oracle_step st;
        st.rung = ids;
        st.f = ds_ini * pow(ds_geo, (double)ids);
        st.tau = st.f * tsamp;
        const double pmax_samples = pmax / st.tau;
        st.n = oracle_downsampled_size(n, st.f);
        size_t bstop = bmax;
        if (st.n < bstop) bstop = st.n;
        if ((size_t)pmax_samples < bstop) bstop = (size_t)pmax_samples;
        for (size_t bins = bmin; bins <= bstop; ++bins) {
            st.bins = bins;
            st.rows = st.n / bins;
            st.stdnoise = (float)sqrt((double)st.rows * oracle_downsampled_variance(n, st.f));
            double pceil = (double)bins + 1.0;
            if (pmax_samples < pceil) pceil = pmax_samples;
            const size_t cs = ceilshift(st.rows, bins, pceil);
            st.rows_eval = st.rows < cs ? st.rows : cs;
            cb(&st, ctx);
        }
    }
}

static void count_cb(const oracle_step* st, void* ctx) { *(size_t*)ctx += st->rows_eval; }

size_t oracle_periodogram_length(size_t n, double tsamp, double pmin, double pmax,
                                 size_t bmin, size_t bmax)
{
    size_t len = 0;
    plan_walk(n, tsamp, pmin, pmax, bmin, bmax, count_cb, &len);
    return len;
}

/* Grid form selector: 1 = form emitted by the reference build
 *   periods[s] = (B*B*tau) / fma(s, -1/(rows-1), B)
 * 0 = source text of periodogram.hpp:192: tau * B * B / (B - s / (rows - 1.0)) */
static int g_grid_emitted = 1;
void oracle_set_grid_emitted(int on) { g_grid_emitted = on; }

typedef struct {
    const float* data;
    size_t size;
    const uint64_t* widths;
    size_t nw;
    double* periods;
    uint32_t* foldbins;
    float* snrs;
    float* ds;    /* downsample buffer */
    float* ffa;   /* ffa output */
    float* tmp;   /* ffa scratch */
    float* cps;
    int grid_only;
} pgram_ctx;

static void pgram_cb(const oracle_step* st, void* vctx)
{
    pgram_ctx* c = (pgram_ctx*)vctx;
    const size_t B = st->bins;
    for (size_t s = 0; s < st->rows_eval; ++s) {
        double per;
        if (g_grid_emitted) {
            const double num = (double)(B * B) * st->tau;
            per = num / fma((double)s, -1.0 / ((double)st->rows - 1.0), (double)B);
        } else {
            per = st->tau * (double)B * (double)B / ((double)B - (double)s / ((double)st->rows - 1.0));
        }
        c->periods[s] = per;
        c->foldbins[s] = (uint32_t)B;
    }
    if (!c->grid_only && st->rows_eval > 0) {
        const float* input = c->data;
        if (!(st->f == 1.0)) {
            /* the ladder re-reads the original series at every rung (periodogram.hpp:162-168) */
            oracle_downsample(c->data, c->size, st->f, c->ds);
            input = c->ds;
        }
        ffa_rec(input, c->tmp, c->ffa, st->rows, B);
        for (size_t s = 0; s < st->rows_eval; ++s)
            snr_row(c->ffa + s * B, B, c->widths, c->nw, st->stdnoise, c->cps, c->snrs + s * c->nw);
    }
    c->periods += st->rows_eval;
    c->foldbins += st->rows_eval;
    c->snrs += st->rows_eval * c->nw;
}

/* Full periodogram (periodogram.hpp:117-201).  Caller validated arguments and
 * widths (0 < w < bins_min).  grid_only != 0 skips downsample/FFA/S/N.
 * Returns -1 on allocation failure. */
int oracle_periodogram(const float* data, size_t size, double tsamp, const uint64_t* widths,
                       size_t nw, double pmin, double pmax, size_t bmin, size_t bmax,
                       double* periods, uint32_t* foldbins, float* snrs, int grid_only)
{
    pgram_ctx c;
    memset(&c, 0, sizeof c);
    c.data = data;
    c.size = size;
    c.widths = widths;
    c.nw = nw;
    c.periods = periods;
    c.foldbins = foldbins;
    c.snrs = snrs;
    c.grid_only = grid_only;
    if (!grid_only) {
        const double ds_ini = pmin / (tsamp * (double)bmin);
        const size_t bufsize = oracle_downsampled_size(size, ds_ini) + 1;
        uint64_t wmax = 0;
        for (size_t i = 0; i < nw; ++i)
            if (widths[i] > wmax) wmax = widths[i];
        c.ds = (float*)malloc(bufsize * sizeof(float));
        c.ffa = (float*)malloc(bufsize * sizeof(float));
        c.tmp = (float*)malloc(bufsize * sizeof(float));
        c.cps = (float*)malloc((bmax + (size_t)wmax + 1) * sizeof(float));
        if (!c.ds || !c.ffa || !c.tmp || !c.cps) {
            free(c.ds); free(c.ffa); free(c.tmp); free(c.cps);
            return -1;
        }
    }
    plan_walk(size, tsamp, pmin, pmax, bmin, bmax, pgram_cb, &c);
    free(c.ds); free(c.ffa); free(c.tmp); free(c.cps);
    return 0;
}

/* The same periodogram on `nthreads` host threads (full-size parity tests:
 * every one of the L x W values of cfg2 against this checker).  Each rung's
 * series is downsampled once; the (rung, bins) steps then run on the threads,
 * each writing its own rows_eval rows of periods / foldbins / snrs.  Per
 * step the arithmetic is pgram_cb's, so the output is identical to
 * oracle_periodogram's for any thread count. */
typedef struct {
    oracle_step* st;
    size_t n, cap;
} step_list;

static void collect_cb(const oracle_step* st, void* ctx)
{
    step_list* l = (step_list*)ctx;
    if (l->n == l->cap) {
        l->cap = l->cap ? 2 * l->cap : 256;
        l->st = (oracle_step*)realloc(l->st, l->cap * sizeof(oracle_step));
    }
    if (l->st) l->st[l->n++] = *st;
}

typedef struct {
    const float* data;
    size_t size;
    const uint64_t* widths;
    size_t nw, bmax, wmax;
    const step_list* steps;
    const size_t* row0;          /* first output row of each step */
    float* const* rung_series;   /* downsampled series of each rung (NULL: f == 1) */
    size_t nrungs;
    double* periods;
    uint32_t* foldbins;
    float* snrs;
    size_t next;                 /* next unit of work (rungs, then steps) */
    pthread_mutex_t mu;
    int phase;                   /* 0: downsample rungs, 1: steps */
    int failed;
} mt_ctx;

static int mt_take(mt_ctx* c, size_t limit, size_t* idx)
{
    pthread_mutex_lock(&c->mu);
    const int ok = c->next < limit;
    if (ok) *idx = c->next++;
    pthread_mutex_unlock(&c->mu);
    return ok;
}

static void* mt_ladder(void* v)
{
    mt_ctx* c = (mt_ctx*)v;
    size_t r;
    while (mt_take(c, c->nrungs, &r)) {
        /* the first step of rung r carries its factor */
        for (size_t i = 0; i < c->steps->n; ++i)
            if (c->steps->st[i].rung == r) {
                const oracle_step* st = &c->steps->st[i];
                if (c->rung_series[r]) oracle_downsample(c->data, c->size, st->f, c->rung_series[r]);
                break;
            }
    }
    return NULL;
}

static void* mt_steps(void* v)
{
    mt_ctx* c = (mt_ctx*)v;
    float* tmp = NULL; float* ffa = NULL; float* cps = NULL;
    size_t i, bufsize = 0;
    for (size_t k = 0; k < c->steps->n; ++k) {
        const size_t cells = c->steps->st[k].rows * c->steps->st[k].bins;
        if (cells > bufsize) bufsize = cells;
    }
    tmp = (float*)malloc((bufsize + 1) * sizeof(float));
    ffa = (float*)malloc((bufsize + 1) * sizeof(float));
    cps = (float*)malloc((c->bmax + c->wmax + 1) * sizeof(float));
    if (!tmp || !ffa || !cps) {
        c->failed = 1;
        free(tmp); free(ffa); free(cps);
        return NULL;
    }
    while (mt_take(c, c->steps->n, &i)) {
        const oracle_step* st = &c->steps->st[i];
        const size_t B = st->bins, r0 = c->row0[i];
        for (size_t s = 0; s < st->rows_eval; ++s) {
            double per;
            if (g_grid_emitted) {
                const double num = (double)(B * B) * st->tau;
                per = num / fma((double)s, -1.0 / ((double)st->rows - 1.0), (double)B);
            } else {
                per = st->tau * (double)B * (double)B / ((double)B - (double)s / ((double)st->rows - 1.0));
            }
            c->periods[r0 + s] = per;
            c->foldbins[r0 + s] = (uint32_t)B;
        }
        if (st->rows_eval == 0) continue;
        const float* input = c->rung_series[st->rung] ? c->rung_series[st->rung] : c->data;
        ffa_rec(input, tmp, ffa, st->rows, B);
        for (size_t s = 0; s < st->rows_eval; ++s)
            snr_row(ffa + s * B, B, c->widths, c->nw, st->stdnoise, cps, c->snrs + (r0 + s) * c->nw);
    }
    free(tmp); free(ffa); free(cps);
    return NULL;
}

int oracle_periodogram_mt(const float* data, size_t size, double tsamp, const uint64_t* widths,
                          size_t nw, double pmin, double pmax, size_t bmin, size_t bmax,
                          double* periods, uint32_t* foldbins, float* snrs, int nthreads)
{
    step_list steps = {NULL, 0, 0};
    plan_walk(size, tsamp, pmin, pmax, bmin, bmax, collect_cb, &steps);
    if (steps.n == 0) return 0;
    if (!steps.st) return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    mt_ctx c;
    memset(&c, 0, sizeof c);
    c.data = data; c.size = size; c.widths = widths; c.nw = nw; c.bmax = bmax;
    for (size_t i = 0; i < nw; ++i)
        if (widths[i] > c.wmax) c.wmax = widths[i];
    c.steps = &steps;
    c.periods = periods; c.foldbins = foldbins; c.snrs = snrs;
    c.nrungs = steps.st[steps.n - 1].rung + 1;
    size_t* row0 = (size_t*)malloc(steps.n * sizeof(size_t));
    float** rs = (float**)calloc(c.nrungs, sizeof(float*));
    int rc = 0;
    if (!row0 || !rs) rc = -1;
    for (size_t i = 0, acc = 0; rc == 0 && i < steps.n; ++i) {
        row0[i] = acc;
        acc += steps.st[i].rows_eval;
        const oracle_step* st = &steps.st[i];
        if (!(st->f == 1.0) && !rs[st->rung]) {
            rs[st->rung] = (float*)malloc((st->n + 1) * sizeof(float));
            if (!rs[st->rung]) rc = -1;
        }
    }
    if (rc == 0) {
        c.row0 = row0;
        c.rung_series = rs;
        pthread_mutex_init(&c.mu, NULL);
        pthread_t th[256];
        for (int phase = 0; phase < 2 && rc == 0; ++phase) {
            c.next = 0;
            int started = 0;
            for (int t = 0; t < nthreads; ++t, ++started)
                if (pthread_create(&th[t], NULL, phase ? mt_steps : mt_ladder, &c) != 0) break;
            if (started == 0) rc = -1;
            for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
            if (c.failed) rc = -1;
        }
        pthread_mutex_destroy(&c.mu);
    }
    if (rs)
        for (size_t r = 0; r < c.nrungs; ++r) free(rs[r]);
    free(rs); free(row0); free(steps.st);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* Running median (running_median.hpp:100-132): exact median of an odd window */
/* with edge replication.  Restated as "k-th order statistic of the window",  */
/* which is what the ring buffer + quickselect returns.                       */
/* ------------------------------------------------------------------------- */
static int cmp_float(const void* a, const void* b)
{
    const float x = *(const float*)a, y = *(const float*)b;
    return (x > y) - (x < y);
}

int oracle_running_median(const float* x, size_t n, size_t width, float* out)
{
    const size_t half = width / 2;
    float* win = (float*)malloc(width * sizeof(float));
    if (!win)
        return -1;
    for (size_t i = 0; i < n; ++i) {
        for (size_t j = 0; j < width; ++j) {
            long long idx = (long long)i - (long long)half + (long long)j;
            if (idx < 0) idx = 0;
            if (idx >= (long long)n) idx = (long long)n - 1;
            win[j] = x[idx];
        }
        qsort(win, width, sizeof(float), cmp_float);
        out[i] = win[half];
    }
    free(win);
    return 0;
}

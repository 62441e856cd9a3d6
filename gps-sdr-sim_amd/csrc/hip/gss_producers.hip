/*
 * gss_producers.hip — the 30 s producers on the GPU: the C/A chip table
 * (codegen, gpssim.c:132-171) and the LNAV frame rows with parity (generateNavMsg,
 * gpssim.c:1467-1547; computeChecksum 693-756) that the render kernels read, built on the device
 * from the host plane's compact sources (gss_nav_src_t).  The arithmetic is gss_nav.h, shared
 * with the host checker gss_nav_rows_host.  gss_run builds its device nav table with them.
 * Also the planner's carrier chain walked ahead: gss_spec_kernel runs each
 * block's walk from a guess of its start (gss_phase.h, speculative block walk), one lane per row,
 * so that the serial chain on the host (gss_carr_chain_spec) takes one partial cycle per block.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gpssim_amd.h"
#include "../common/gss_nav.h"
#include "../common/gss_phase.h"

extern "C" int gss_fail(int code, const char *fmt, ...);
extern "C" int gss_dev_ordinal(const gss_dev *d);

/* one workgroup of 64 lanes: lane 0 runs the two 10-stage registers (1023 steps), then the wave
   forms each PRN's chips 64 at a time and packs them with a ballot */
__global__ __launch_bounds__(64) void gss_ca_kernel(uint32_t *__restrict__ out)
{
    __shared__ uint32_t g1[GSS_CA_WORDS], g2[GSS_CA_WORDS];
    const int lane = threadIdx.x;
    if (lane == 0)
        gss_g1g2(g1, g2);
    __syncthreads();
    for (int prn = 1; prn <= 32; prn++)
        for (int c0 = 0; c0 < 32 * GSS_CA_WORDS; c0 += 64) {
            const int i = c0 + lane;
            const uint32_t bit = i < GSS_CA_LEN ? gss_ca_chip(g1, g2, prn, i) : 0u;
            const uint64_t m = __builtin_amdgcn_ballot_w64(bit != 0);
            if (lane < 2)
                out[(size_t)(prn - 1) * GSS_CA_WORDS + c0 / 32 + lane] =
                    (uint32_t)(m >> (32 * lane));
        }
}

/* rows [first, first + n): a lane per row whose predecessor is not among them (a chain head)
   builds its row and then the rows that continue it, in order */
__global__ void gss_nav_kernel(const gss_nav_src_t *__restrict__ src, int first, int n,
                               uint32_t *__restrict__ rows)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    if (src[i].prev >= first)
        return;                                   /* built by its chain's head */
    for (int r = first + i, guard = 0; r >= first && r < first + n && guard < n; guard++) {
        const gss_nav_src_t *q = &src[r - first];
        gss_nav_frame(q, gss_nav_head(q, rows), rows + (size_t)r * GSS_NAV_WORDS);
        r = q->next;
    }
}

extern "C" int gss_ca_table_device(gss_dev *d, uint32_t *out, void *stream)
{
    if (!d || !out)
        return gss_fail(GSS_E_ARG, "invalid C/A table arguments");
    if (hipSetDevice(gss_dev_ordinal(d)) != hipSuccess)
        return gss_fail(GSS_E_HIP, "hipSetDevice failed");
    hipLaunchKernelGGL(gss_ca_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "C/A kernel: %s", hipGetErrorString(e));
}

extern "C" int gss_nav_rows_device(gss_dev *d, const gss_nav_src_t *src, int first, int n,
                                   uint32_t *rows, void *stream)
{
    if (!d || (n > 0 && (!src || !rows)) || first < 0 || n < 0)
        return gss_fail(GSS_E_ARG, "invalid nav-row arguments");
    if (n == 0)
        return 0;
    if (hipSetDevice(gss_dev_ordinal(d)) != hipSuccess)
        return gss_fail(GSS_E_HIP, "hipSetDevice failed");
    hipLaunchKernelGGL(gss_nav_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0,
                       (hipStream_t)stream, src, first, n, rows);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "nav kernel: %s", hipGetErrorString(e));
}

/* one lane per segment of a row (gss_spec_seg_walk).  Rows laid out [nblk][GSS_MAXCH] are taken
   channel-major, so that a wave's lanes walk the segments of consecutive blocks of one channel:
   close steps, nearly the same cycles and binades (uniform control flow) instead of 16 different
   Dopplers per wave.
   The rows and walks live in pinned host memory (gss_run), so the workgroup (8 rows x 8
   segments) stages them in LDS: each row read once across the link in 8-byte words instead of
   by each of its 8 lanes, and the walks written back whole (16-byte stores, 272 B per row)
   instead of field by field -- the walks' link traffic had slowed the slot downloads beside
   them by a tenth (tools/d2h_overlap.py).  Segments past a row's k are written as zeros. */
constexpr int SPEC_ROWS = 64 / GSS_SPEC_K;               /* rows per workgroup */
static_assert(sizeof(gss_spec_in_t) % 8 == 0 && sizeof(gss_spec_t) % 16 == 0, "row sizes");

__device__ inline int spec_row_of(int u, int nrow)
{
    const int nb = nrow / GSS_MAXCH;
    return nrow % GSS_MAXCH ? u : (u % nb) * GSS_MAXCH + u / nb;
}

/* ---- a cycle cache shared by the GSS_SPEC_K lanes of one row, in LDS ----------------------------
 * The 8 segments of a row walk with the same step s, so every cycle map one lane walks (its
 * start interval [lo, hi], length L, end v0 of start w0: gss_cc_put's entry) serves the other
 * seven too.  Each lane writes its own 4 entries (a ring), every lane reads all 32; all of a
 * row's lanes are in one wave, so a lane's LDS writes are seen by the wave's later reads (program
 * order), no barrier.  A per-lane cache (GSS_SPEC_CC) missed at each lane's own cycles, so the
 * wave walked nearly every cycle in full (12 % slower than no cache); shared, a row's cache holds
 * its ~10-16 cycle types after each lane's first few cycles and the wave then mostly takes the
 * O(1) path.  The intervals are the cached walks' (shrunk by `safe`), so a segment's [dlo, dhi]
 * can be narrower than the host's plain walk (gss_walk_margins) gives: still conservative, the
 * same ends and wraps, and the chain exact (tests/test_gpu_parity.py test_spec_records_on_device). */
constexpr int SCC_PER_LANE = 4;
constexpr int SCC_N = GSS_SPEC_K * SCC_PER_LANE;         /* entries per row */
struct spec_cc {
    double lo[SCC_N], hi[SCC_N], w0[SCC_N], v0[SCC_N];
    int32_t L[SCC_N];                                    /* 0: empty */
    int32_t succ[SCC_N];                                 /* the entry the next cycle used */
};

/* an entry holding start w with at most nmax steps, the hint (the successor of the previous
   cycle's entry) first; -1 if none.  The entry is copied out in the same reads that test it: a
   lane on the other side of a divergent branch may overwrite the slot (its ring) before this
   lane uses it */
struct scc_entry {
    double lo, hi, w0, v0;
    int32_t L;
};
__device__ inline bool scc_take(const spec_cc *c, int i, double w, int64_t nmax, scc_entry *h)
{
    const int32_t L = c->L[i];
    const double lo = c->lo[i], hi = c->hi[i], w0 = c->w0[i], v0 = c->v0[i];
    if (!(L > 0 && w >= lo && w <= hi && L <= nmax))
        return false;
    *h = scc_entry{lo, hi, w0, v0, L};
    return true;
}
__device__ inline int scc_find(const spec_cc *c, double w, int64_t nmax, int prev, scc_entry *h)
{
    if (prev >= 0) {
        const int p = c->succ[prev];
        if (p >= 0 && scc_take(c, p, w, nmax, h))
            return p;
    }
    for (int i = 0; i < SCC_N; i++)
        if (scc_take(c, i, w, nmax, h))
            return i;
    return -1;
}

__device__ inline int scc_put(spec_cc *c, int j, int &ring, double w, double dlo, double dhi,
                              double safe, double v_end, int64_t L)
{
    if (!(dlo <= 0.0 && dhi >= 0.0) || L <= 0 || L > INT32_MAX)
        return -1;
    const int i = j * SCC_PER_LANE + (ring++ & (SCC_PER_LANE - 1));
    double lo = w + dlo + safe, hi = w + dhi - safe;
    if (lo > w) lo = w;                                  /* the walked start is always valid */
    if (hi < w) hi = w;
    c->L[i] = 0;                                         /* (invalid while rewritten) */
    c->lo[i] = lo;
    c->hi[i] = hi;
    c->w0[i] = w;
    c->v0[i] = v_end;
    c->succ[i] = -1;
    c->L[i] = (int32_t)L;
    return i;
}

/* gss_walk_margins from a post-wrap value x, whole cycles from the row's shared cache */
__device__ double spec_walk_margins_shared(double x, double s, int64_t n, double *dlo,
                                           double *dhi, int *wrap_end, spec_cc *c, int j)
{
    int64_t left = n;
    int last = 0, prev = -1, ring = 0;
    const double safe = 4.0 * gss_pow2(-52);
    const double T = s > 0.0 ? 0.0 : gss_pow2(gss_exp2i(-s) + 2);
    const double dunit = gss_pow2(-53);
    while (left > 0) {
        const double w = x;
        scc_entry h;
        const int e = scc_find(c, w, left, prev, &h);
        if (prev >= 0 && e >= 0)
            c->succ[prev] = e;
        if (e >= 0) {
            const double lo = h.lo - w, hi = h.hi - w;
            if (lo > *dlo) *dlo = lo;
            if (hi < *dhi) *dhi = hi;
            x = h.v0 + (w - h.w0);
            left -= h.L;
            prev = e;
            if (s > 0.0) {
                last = 1;
                continue;
            }
        } else {
            double clo = -GSS_BIG, chi = GSS_BIG;
            int st = 0;
            int64_t taken;
            if (s > 0.0) {
                taken = gss_asc_to_wrap(&x, s, 1.0, left, &st, &clo, &chi);
                last = st;
            } else {
                last = 0;
                taken = gss_desc_head(&x, s, T, left, &st, &clo, &chi);
            }
            left -= taken;
            if (clo > *dlo) *dlo = clo;
            if (chi < *dhi) *dhi = chi;
            const int put = st ? scc_put(c, j, ring, w, clo, chi, safe, x, taken) : -1;
            if (prev >= 0 && put >= 0)
                c->succ[prev] = put;
            prev = put;
            if (s > 0.0)
                continue;
            if (!st || left <= 0)
                break;
        }
        last = 0;
        while (left > 0) {                      /* descending, below T: real steps to the wrap */
            gss_margin_step(x, s, dunit, dlo, dhi);
            const double r = x + s;
            left--;
            if (r < 0.0) {
                const double lim = -r - 2.0 * dunit;
                if (lim < *dhi) *dhi = lim;
                gss_margin_step(r, 1.0, dunit, dlo, dhi);
                x = r + 1.0;
                last = 1;
                break;
            }
            if (-r > *dlo) *dlo = -r;
            x = r;
        }
    }
    *wrap_end = last;
    return x;
}

/* gss_spec_seg_walk (gss_phase.h) with the segment's margins walk from the row's shared cache */
__device__ void spec_seg_walk_shared(const gss_spec_in_t *in, int j, int64_t n, gss_spec_t *o,
                                     spec_cc *c)
{
    const double s = in->s;
    const int k = in->k < 1 ? 1 : (in->k > GSS_SPEC_K ? GSS_SPEC_K : in->k);
    gss_spec_seg_t *sg = &o->seg[j];
    const int64_t stop = j + 1 < k ? in->P[j + 1] : n;
    double x;
    int64_t pos;
    sg->dlo = 1.0;
    sg->dhi = 0.0;
    sg->wrap_end = 0;
    if (j == 0) {
        x = in->g;
        int wr = 0;
        const int64_t t = s != 0.0 ? gss_carr_to_wrap(&x, s, stop, &wr) : stop;
        o->p1 = wr ? t : n;
        o->w1 = x;
        sg->end = x;
        if (!wr || t >= stop)
            return;
        pos = t;
    } else {
        x = in->W[j];
        pos = in->P[j];
        sg->end = x;
        if (s == 0.0 || pos >= stop)
            return;
    }
    double dlo = -GSS_BIG, dhi = GSS_BIG;
    int we = 0;
    x = spec_walk_margins_shared(x, s, stop - pos, &dlo, &dhi, &we, c, j);
    sg->end = x;
    sg->dlo = dlo;
    sg->dhi = dhi;
    sg->wrap_end = we;
}

/* in: the rows (read); back: where the rows go back with the walkers' guesses (in itself for
   gss_spec_device, only the rows guessed here; the device copy for gss_spec_records_device, every
   row).  heads: read only each row's start, step, k and pad (the walkers guess the rest) */
__global__ __launch_bounds__(64) void gss_spec_kernel(const gss_spec_in_t *in,
                                                      gss_spec_in_t *back, int nrow, int n,
                                                      gss_spec_t *__restrict__ spec, int heads)
{
    __shared__ gss_spec_in_t s_in[SPEC_ROWS];
    __shared__ gss_spec_t s_out[SPEC_ROWS];
    __shared__ int s_guessed[SPEC_ROWS];
    __shared__ spec_cc s_cc[SPEC_ROWS];                  /* a cycle cache per row */
    constexpr int WI = sizeof(gss_spec_in_t) / 8, WO = sizeof(gss_spec_t) / 16;
    const int lane = threadIdx.x, r = lane / GSS_SPEC_K, j = lane % GSS_SPEC_K;
    const int u0 = blockIdx.x * SPEC_ROWS;
    const int wr = heads ? 3 : WI;                       /* g, s, (k, pad): 3 words */
    for (int q = lane; q < SPEC_ROWS * WI; q += 64) {    /* the rows in, 8 bytes a lane */
        const int rr = q / WI, w = q % WI;
        if (u0 + rr < nrow)
            ((uint64_t *)&s_in[rr])[w] =
                w < wr ? ((const uint64_t *)&in[spec_row_of(u0 + rr, nrow)])[w] : 0;
    }
    for (int q = lane; q < SPEC_ROWS * WO; q += 64)      /* the walks zeroed */
        ((uint4 *)s_out)[q] = make_uint4(0, 0, 0, 0);
    for (int q = lane; q < SPEC_ROWS * SCC_N; q += 64)   /* the caches empty */
        s_cc[q / SCC_N].L[q % SCC_N] = 0;
    __syncthreads();
    const bool live = u0 + r < nrow;
    gss_spec_in_t row = s_in[r];
    const bool guess = live && row.k == 0;
    if (guess) {
        /* segment starts not guessed yet (gss_carr_chain_starts): every lane of the row makes
           the same guesses; its first lane writes them back for the host's chain */
        gss_spec_guess_row(row.g, row.s, n, &row);
    }
    __syncthreads();                                     /* every lane has read s_in[r] */
    if (j == 0) {
        s_guessed[r] = guess;
        if (guess)
            s_in[r] = row;
    }
    if (live && j < row.k)
        spec_seg_walk_shared(&row, j, n, &s_out[r], &s_cc[r]);
    __syncthreads();
    for (int q = lane; q < SPEC_ROWS * WO; q += 64) {    /* the walks out, 16 bytes a lane */
        const int rr = q / WO, w = q % WO;
        if (u0 + rr < nrow)
            ((uint4 *)&spec[spec_row_of(u0 + rr, nrow)])[w] = ((const uint4 *)&s_out[rr])[w];
    }
    for (int q = lane; q < SPEC_ROWS * WI; q += 64) {    /* the walkers' guesses back */
        const int rr = q / WI, w = q % WI;
        if (u0 + rr < nrow && (s_guessed[rr] || back != in))
            ((uint64_t *)&back[spec_row_of(u0 + rr, nrow)])[w] = ((const uint64_t *)&s_in[rr])[w];
    }
}

/* Each row's record (gss_phase.h gss_spec_record) from the walks in device memory: one lane per
   row, the link from the previous row of its slot (in[].pad); the records staged in LDS and
   written to host-visible memory in 16-byte stores (72 B per row instead of the walk's 272 and
   the guesses' 152) */
constexpr int REC_ROWS = 64;
static_assert(sizeof(gss_spec_rec_t) == 72, "record size");

__global__ __launch_bounds__(REC_ROWS) void gss_spec_rec_kernel(
    const gss_spec_in_t *__restrict__ in, const gss_spec_t *__restrict__ spec, int nrow, int n,
    gss_spec_rec_t *__restrict__ rec)
{
    __shared__ gss_spec_rec_t s_rec[REC_ROWS];
    const int lane = threadIdx.x;
    const int u0 = blockIdx.x * REC_ROWS, i = u0 + lane;
    if (i < nrow) {
        const int p = in[i].pad;
        const bool ok = p >= 0 && p < i;
        gss_spec_record(&in[i], &spec[i], ok ? &in[p] : nullptr, ok ? &spec[p] : nullptr, n,
                        &s_rec[lane]);
        if (s_rec[lane].ok & 2)
            s_rec[lane].ok |= (i - p) << 2;         /* the row the link was built against */
    }
    __syncthreads();
    constexpr int W = sizeof(gss_spec_rec_t) * REC_ROWS / 16;
    const int rows = nrow - u0 < REC_ROWS ? nrow - u0 : REC_ROWS;
    const int words = rows * (int)sizeof(gss_spec_rec_t) / 8;   /* 9 words a row */
    if (rows == REC_ROWS) {
        for (int q = lane; q < W; q += REC_ROWS)
            ((uint4 *)&rec[u0])[q] = ((const uint4 *)s_rec)[q];
    } else {
        for (int q = lane; q < words; q += REC_ROWS)
            ((uint64_t *)&rec[u0])[q] = ((const uint64_t *)s_rec)[q];
    }
}

extern "C" int gss_spec_records_device(gss_dev *d, const gss_spec_in_t *in, int nrow,
                                       int n_per_blk, gss_spec_in_t *d_in, gss_spec_t *d_spec,
                                       gss_spec_rec_t *rec, void *stream)
{
    if (!d || nrow < 0 || n_per_blk <= 0 ||
        (nrow > 0 && (!in || !d_in || !d_spec || !rec)) || ((uintptr_t)in & 7) ||
        ((uintptr_t)d_in & 7) || ((uintptr_t)d_spec & 15) || ((uintptr_t)rec & 15) ||
        (const void *)in == (const void *)d_in)
        return gss_fail(GSS_E_ARG, "invalid speculative-record arguments (rows 8-byte, walks "
                        "and records 16-byte aligned, in and d_in apart)");
    if (nrow == 0)
        return 0;
    if (hipSetDevice(gss_dev_ordinal(d)) != hipSuccess)
        return gss_fail(GSS_E_HIP, "hipSetDevice failed");
    hipLaunchKernelGGL(gss_spec_kernel, dim3((unsigned)((nrow + SPEC_ROWS - 1) / SPEC_ROWS)),
                       dim3(64), 0, (hipStream_t)stream, in, d_in, nrow, n_per_blk, d_spec, 1);
    hipLaunchKernelGGL(gss_spec_rec_kernel, dim3((unsigned)((nrow + REC_ROWS - 1) / REC_ROWS)),
                       dim3(REC_ROWS), 0, (hipStream_t)stream, d_in, d_spec, nrow, n_per_blk,
                       rec);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "record kernels: %s", hipGetErrorString(e));
}

extern "C" int gss_spec_device(gss_dev *d, gss_spec_in_t *in, int nrow, int n_per_blk,
                               gss_spec_t *spec, void *stream)
{
    if (!d || nrow < 0 || n_per_blk <= 0 || (nrow > 0 && (!in || !spec)) ||
        ((uintptr_t)in & 7) || ((uintptr_t)spec & 15))
        return gss_fail(GSS_E_ARG, "invalid speculative-walk arguments (rows 8-byte, walks "
                        "16-byte aligned)");
    if (nrow == 0)
        return 0;
    if (hipSetDevice(gss_dev_ordinal(d)) != hipSuccess)
        return gss_fail(GSS_E_HIP, "hipSetDevice failed");
    hipLaunchKernelGGL(gss_spec_kernel, dim3((unsigned)((nrow + SPEC_ROWS - 1) / SPEC_ROWS)),
                       dim3(64), 0,
                       (hipStream_t)stream, in, in, nrow, n_per_blk, spec, 0);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "spec kernel: %s", hipGetErrorString(e));
}

/* gss_run's uploads of its slots' inputs (gss_run.hip, dev_copy): 16-byte vector loads, four in
   flight per lane; the tail bytes (and unaligned buffers) byte by byte */
__global__ __launch_bounds__(256) void upload_kernel(const uint4 *__restrict__ src,
                                                     uint4 *__restrict__ dst, size_t n16,
                                                     int tail)
{
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride],
                    d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride)
        dst[i] = src[i];
    if (blockIdx.x == 0 && (int)threadIdx.x < tail)
        ((uint8_t *)(dst + n16))[threadIdx.x] = ((const uint8_t *)(src + n16))[threadIdx.x];
}

__global__ __launch_bounds__(256) void upload_bytes_kernel(const uint8_t *__restrict__ src,
                                                           uint8_t *__restrict__ dst, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        dst[i] = src[i];
}

/* n bytes from src to dst by a kernel on st: pinned host (hipHostMalloc) or device memory on
   either side (gss_run's uploads; not exported) */
int run_copy_launch(void *dst, const void *src, size_t n, hipStream_t st)
{
    if (n == 0)
        return 0;
    if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
        const size_t n16 = n >> 4;
        const size_t g = (n16 + 1023) / 1024;
        hipLaunchKernelGGL(upload_kernel, dim3((unsigned)(g < 1 ? 1 : g > 2048 ? 2048 : g)),
                           dim3(256), 0, st, (const uint4 *)src, (uint4 *)dst, n16,
                           (int)(n & 15));
    } else {
        const size_t g = (n + 255) / 256;
        hipLaunchKernelGGL(upload_bytes_kernel, dim3((unsigned)(g > 2048 ? 2048 : g)), dim3(256),
                           0, st, (const uint8_t *)src, (uint8_t *)dst, n);
    }
    return hipGetLastError() == hipSuccess ? 0 : gss_fail(GSS_E_HIP, "copy kernel launch");
}

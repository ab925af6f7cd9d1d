/*
 * sgbm_oracle.c -- CPU restatement of OpenCV 4.6.0 StereoSGBM / medianBlur(3) / filterSpeckles /
 * reprojectImageTo3D / BGR2GRAY / INTER_AREA 0.5x.  TEST INFRASTRUCTURE ONLY (see sgbm_oracle.h:
 * parity against real OpenCV is UNPINNED; the oracle is pinned by known-answer tests and by
 * independent numpy/scipy restatements in tests/test_oracle_*.py).
 *
 * The loop structure deliberately mirrors the OpenCV drivers (row-by-row, ring buffers, running
 * sums, the same border rules) rather than the GPU engine's formulation, so that GPU-vs-oracle
 * agreement is evidence about the algorithm and not a restatement compared with itself.
 *
 * Section map:
 *   A.1/A.2  prefilter + Birchfield-Tomasi  -> calc_pixel_cost_bt()
 *   A.3      block sum (running sums)       -> sgbm_rows() / sgbm3way_stripe()
 *   A.4-A.6  path recurrence, MODE_SGBM/HH  -> sgbm_rows()
 *   A.7      MODE_SGBM_3WAY stripes         -> sgbm3way()
 *   A.8/A.9  WTA/uniqueness/subpixel/LR     -> wta_pixel(), lr_check_row()
 *   A.10     medianBlur 3x3                 -> orc_median3x3_s16()
 *   A.11     filterSpeckles                 -> orc_filter_speckles_s16()
 *   A.12     reprojectImageTo3D             -> orc_reproject_f32()
 *   A.13     BGR2GRAY, INTER_AREA, 1/16     -> orc_bgr2gray(), orc_resize_area_half(), ...
 *
 * Build: gcc -O2 -ffp-contract=off (contraction must stay off: reprojection parity is bitwise).
 */
#include "sgbm_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

typedef int16_t cost_t;

#define DISP_SHIFT 4
#define DISP_SCALE 16
#define MAX_COST 32767
#define TAB_OFS 1024

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline cost_t sat16(int v) { return (cost_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v)); }

/* ------------------------------------------------------------------------------------------ */
/* Effective parameters, with OpenCV's defaulting rules (stereosgbm.cpp computeDisparitySGBM /  */
/* SGBM3WayMainLoop constructor).                                                              */
/* ------------------------------------------------------------------------------------------ */
typedef struct eff_params {
    int minD, maxD, D, width1, minX1, maxX1;
    int SW2, SH2;
    int P1, P2;
    int uniq, disp12MaxDiff, ftzero;
    int uniq_simd;
    int invalid_scaled;
    int cn;  /* interleaved channels of the input images (1 or 3) */
} eff_params;

static int make_eff(const orc_params* p, int width, eff_params* e)
{
    if (p->numDisparities <= 0 || (p->numDisparities % 16) != 0) return -2;
    e->minD = p->minDisparity;
    e->D = p->numDisparities;
    e->maxD = e->minD + e->D;
    e->minX1 = imax(e->maxD, 0);
    e->maxX1 = width + imin(e->minD, 0);
    e->width1 = e->maxX1 - e->minX1;
    if (p->mode == ORC_MODE_SGBM_3WAY) {
        /* SGBM3WayMainLoop: SW2 = SH2 = SADWindowSize > 0 ? SADWindowSize/2 : 1 */
        e->SW2 = e->SH2 = p->blockSize > 0 ? p->blockSize / 2 : 1;
    } else {
        /* calcSADWindowSize(): SADWindowSize > 0 ? SADWindowSize : 5 */
        int bs = p->blockSize > 0 ? p->blockSize : 5;
        e->SW2 = e->SH2 = bs / 2;
    }
    e->P1 = p->P1 > 0 ? p->P1 : 2;
    e->P2 = imax(p->P2 > 0 ? p->P2 : 5, e->P1 + 1);
    e->uniq = p->uniquenessRatio >= 0 ? p->uniquenessRatio : 10;
    e->disp12MaxDiff = p->disp12MaxDiff > 0 ? p->disp12MaxDiff : 1;
    e->ftzero = imax(p->preFilterCap, 15) | 1;
    if (p->uniq_rule == ORC_UNIQ_SCALAR) e->uniq_simd = 0;
    else if (p->uniq_rule == ORC_UNIQ_SIMD) e->uniq_simd = 1;
    else e->uniq_simd = (p->mode == ORC_MODE_SGBM_3WAY);
    e->invalid_scaled = (e->minD - 1) * DISP_SCALE;
    e->cn = 1;
    return 0;
}

static void make_clip_tab(int ftzero, uint8_t* tab /* TAB_OFS*2 + 256 */)
{
    for (int k = 0; k < TAB_OFS * 2 + 256; k++) {
        int v = k - TAB_OFS;
        v = v < -ftzero ? -ftzero : (v > ftzero ? ftzero : v);
        tab[k] = (uint8_t)(v + ftzero);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* A.1 + A.2: calcPixelCostBT for one image row y of an 8-bit image with cn (1 or 3)           */
/* interleaved channels.  Prefiltered channels 0..cn-1 are the per-channel x-Sobels (cost      */
/* shift 0), cn..2cn-1 the raw channels (cost shift 2); the pixel cost sums all 2cn of them.   */
/* cost: [width1][D], cost[(x-minX1)*D + (d-minD)] for x in [minX1,maxX1), d in [minD,maxD).   */
/* ------------------------------------------------------------------------------------------ */
static void calc_pixel_cost_bt(const uint8_t* img1, const uint8_t* img2, size_t step, int width,
                               int height, int y, int minD, int maxD, cost_t* cost,
                               const uint8_t* tab /* centred at 0 */,
                               uint8_t* work /* (4*cn + 2) * width */, int cn)
{
    const int D = maxD - minD;
    const int minX1 = imax(maxD, 0), maxX1 = width + imin(minD, 0);
    const int width1 = maxX1 - minX1;
    const int minX2 = imax(minX1 - maxD, 0), maxX2 = imin(maxX1 - minD, width);

    uint8_t* pre1 = work;                        /* [2cn][width] prefiltered left channels  */
    uint8_t* pre2 = work + 2 * cn * width;       /* [2cn][width] prefiltered right channels */
    uint8_t* v0b = work + 4 * cn * width;        /* min(v, v half-left, v half-right) for the right row */
    uint8_t* v1b = work + (4 * cn + 1) * width;  /* max(...)                                           */

    const uint8_t* r1 = img1 + (size_t)y * step;
    const uint8_t* r2 = img2 + (size_t)y * step;
    /* replicated neighbour rows (n1 = y>0 ? -step : 0, s1 = y<rows-1 ? step : 0) */
    const uint8_t* n1 = y > 0 ? r1 - step : r1;
    const uint8_t* s1 = y < height - 1 ? r1 + step : r1;
    const uint8_t* n2 = y > 0 ? r2 - step : r2;
    const uint8_t* s2 = y < height - 1 ? r2 + step : r2;

    for (int c = 0; c < cn; c++) {
        uint8_t* sob1 = pre1 + c * width;
        uint8_t* raw1 = pre1 + (cn + c) * width;
        uint8_t* sob2 = pre2 + c * width;
        uint8_t* raw2 = pre2 + (cn + c) * width;
        /* columns 0 and width-1 of every prefiltered channel (Sobel and raw) hold tab[0] */
        sob1[0] = sob1[width - 1] = raw1[0] = raw1[width - 1] = tab[0];
        sob2[0] = sob2[width - 1] = raw2[0] = raw2[width - 1] = tab[0];
        for (int x = 1; x < width - 1; x++) {
            const int a = (x + 1) * cn + c, b = (x - 1) * cn + c;
            sob1[x] = tab[(r1[a] - r1[b]) * 2 + n1[a] - n1[b] + s1[a] - s1[b]];
            sob2[x] = tab[(r2[a] - r2[b]) * 2 + n2[a] - n2[b] + s2[a] - s2[b]];
            raw1[x] = r1[x * cn + c];
            raw2[x] = r2[x * cn + c];
        }
    }

    for (int i = 0; i < width1 * D; i++) cost[i] = 0;

    for (int c = 0; c < 2 * cn; c++) {
        const uint8_t* p1 = pre1 + c * width;
        const uint8_t* p2 = pre2 + c * width;
        const int diff_scale = c < cn ? 0 : 2;

        /* half-sample envelope of the right row over the columns the matches can touch */
        for (int xr = minX2; xr < maxX2; xr++) {
            int v = p2[xr];
            int va = xr < width - 1 ? (v + p2[xr + 1]) / 2 : v;
            int vb = xr > 0 ? (v + p2[xr - 1]) / 2 : v;
            int lo = imin(imin(va, vb), v), hi = imax(imax(va, vb), v);
            v0b[xr] = (uint8_t)lo;
            v1b[xr] = (uint8_t)hi;
        }
        for (int x = minX1; x < maxX1; x++) {
            int u = p1[x];
            int ul = x > 0 ? (u + p1[x - 1]) / 2 : u;
            int ur = x < width - 1 ? (u + p1[x + 1]) / 2 : u;
            int u0 = imin(imin(ul, ur), u), u1 = imax(imax(ul, ur), u);
            cost_t* cx = cost + (size_t)(x - minX1) * D;
            for (int d = minD; d < maxD; d++) {
                int xr = x - d;
                int v = p2[xr], v0 = v0b[xr], v1 = v1b[xr];
                int c0 = imax(0, imax(u - v1, v0 - u));
                int c1 = imax(0, imax(v - u1, u0 - v));
                cx[d - minD] = (cost_t)(cx[d - minD] + (imin(c0, c1) >> diff_scale));
            }
        }
    }
}

/* horizontal box sum of one pixel-cost row into hsum (running sum, replicate in [0,width1)) */
static void hsum_row(const cost_t* pix, cost_t* hsum, int width1, int D, int SW2)
{
    for (int d = 0; d < D; d++) {
        int v = pix[d] * (SW2 + 1);
        for (int k = 1; k <= SW2; k++) v += pix[(size_t)imin(k, width1 - 1) * D + d];
        hsum[d] = (cost_t)v;
    }
    for (int x = 1; x < width1; x++) {
        const cost_t* add = pix + (size_t)imin(x + SW2, width1 - 1) * D;
        const cost_t* sub = pix + (size_t)imax(x - SW2 - 1, 0) * D;
        for (int d = 0; d < D; d++)
            hsum[(size_t)x * D + d] = (cost_t)(hsum[(size_t)(x - 1) * D + d] + add[d] - sub[d]);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* A.4 path recurrence for one pixel and one direction.                                        */
/*   L(p,d) = C(p,d) + min(Lp[d], Lp[d-1]+P1, Lp[d+1]+P1, minLp+P2) - (minLp+P2)               */
/* Lp is D+2 long with Lp[0] = Lp[D+1] = MAX_COST sentinels (d = -1 and d = D).                */
/* ------------------------------------------------------------------------------------------ */
static inline int path_step(const cost_t* Cp, const cost_t* Lp /* points at d=0 */, int minLp,
                            cost_t* Lout, int D, int P1, int P2)
{
    const int delta = minLp + P2;
    int minL = MAX_COST;
    for (int d = 0; d < D; d++) {
        int a = Lp[d];
        int b = imin(Lp[d - 1] + P1, Lp[d + 1] + P1);
        int L = Cp[d] + imin(imin(a, b), delta) - delta;
        Lout[d] = (cost_t)L;
        if (L < minL) minL = L;
    }
    return minL;
}

/* A.8: winner-take-all, uniqueness, disp2 candidate, subpixel.  Returns 1 if the pixel is      */
/* accepted (and fills *minS_out, *best_out, *disp16_out), 0 if uniqueness rejected it.        */
static int wta_pixel(const cost_t* Sp, const eff_params* e, int* minS_out, int* best_out,
                     int* disp16_out)
{
    const int D = e->D;
    int minS = MAX_COST, best = -1;
    for (int d = 0; d < D; d++)
        if (Sp[d] < minS) { minS = Sp[d]; best = d; }
    if (e->uniq > 0 || !e->uniq_simd) {
        int d;
        if (e->uniq_simd) {
            /* SGBM3WayMainLoop SIMD rule: cost < (short)(thresh+1), thresh=(100*min)/(100-u) */
            int thresh = (100 * minS) / (100 - e->uniq);
            int16_t tr = (int16_t)(thresh + 1);
            for (d = 0; d < D; d++)
                if (Sp[d] < tr && abs(d - best) > 1) break;
        } else {
            for (d = 0; d < D; d++)
                if (Sp[d] * (100 - e->uniq) < minS * 100 && abs(best - d) > 1) break;
        }
        if (d < D) return 0;
    }
    int d = best;
    *minS_out = minS;
    *best_out = best;
    if (0 < d && d < D - 1) {
        int denom2 = imax(Sp[d - 1] + Sp[d + 1] - 2 * Sp[d], 1);
        d = d * DISP_SCALE + ((Sp[d - 1] - Sp[d + 1]) * DISP_SCALE + denom2) / (denom2 * 2);
    } else {
        d *= DISP_SCALE;
    }
    *disp16_out = d + e->minD * DISP_SCALE;
    return 1;
}

/* A.9: left-right check of one output row against its disp2 (right-view WTA) buffer. */
static void lr_check_row(int16_t* drow, const int16_t* disp2, int width, const eff_params* e)
{
    for (int x = e->minX1; x < e->maxX1; x++) {
        int d1 = drow[x];
        if (d1 == e->invalid_scaled) continue;
        int _d = d1 >> DISP_SHIFT;
        int d_ = (d1 + DISP_SCALE - 1) >> DISP_SHIFT;
        int _x = x - _d, x_ = x - d_;
        if (0 <= _x && _x < width && disp2[_x] >= e->minD && abs(disp2[_x] - _d) > e->disp12MaxDiff &&
            0 <= x_ && x_ < width && disp2[x_] >= e->minD && abs(disp2[x_] - d_) > e->disp12MaxDiff)
            drow[x] = (int16_t)e->invalid_scaled;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* A.3-A.6: computeDisparitySGBM (MODE_SGBM: 5 paths, one pass; MODE_HH: 8 paths, two passes). */
/* ------------------------------------------------------------------------------------------ */
#define NDIR 4

typedef struct lr_bufs {
    /* Lr[buf][x+1][dir][d+1]: x in [-1, width1], d in [-1, D] */
    cost_t* L;
    int* minL; /* minL[buf][x+1][dir] */
    int W1, D;
} lr_bufs;

static inline cost_t* lr_at(const lr_bufs* b, int buf, int x, int dir)
{
    return b->L + ((((size_t)buf * (b->W1 + 2) + (x + 1)) * NDIR + dir) * (b->D + 2)) + 1;
}
static inline int* minl_at(const lr_bufs* b, int buf, int x, int dir)
{
    return b->minL + (((size_t)buf * (b->W1 + 2) + (x + 1)) * NDIR + dir);
}
static void lr_clear(lr_bufs* b)
{
    size_t n = (size_t)2 * (b->W1 + 2) * NDIR;
    for (size_t i = 0; i < n; i++) {
        cost_t* l = b->L + i * (b->D + 2);
        for (int d = 0; d < b->D + 2; d++) l[d] = 0;
        l[0] = l[b->D + 1] = MAX_COST; /* the sentinels OpenCV writes before every read */
        b->minL[i] = 0;
    }
}

/* Fills C rows exactly as the SGBM driver does (pass 1). C is [H][W1][D] when fullDP, else one */
/* row; the callback-free structure keeps the running sums identical to OpenCV.                 */
typedef struct cost_state {
    cost_t* hsum;     /* (2*SH2+2) rows */
    cost_t* pix;      /* one row */
    uint8_t* work;
    uint8_t tab[TAB_OFS * 2 + 256];
    int nrows;
} cost_state;

static int cost_state_init(cost_state* cs, const eff_params* e, int width)
{
    cs->nrows = e->SH2 * 2 + 2;
    size_t row = (size_t)e->width1 * e->D;
    cs->hsum = (cost_t*)calloc(row * cs->nrows, sizeof(cost_t));
    cs->pix = (cost_t*)calloc(row, sizeof(cost_t));
    cs->work = (uint8_t*)calloc((size_t)width * (4 * e->cn + 2), 1);
    make_clip_tab(e->ftzero, cs->tab);
    return (cs->hsum && cs->pix && cs->work) ? 0 : -1;
}
static void cost_state_free(cost_state* cs)
{
    free(cs->hsum); free(cs->pix); free(cs->work);
}

/* One row of the running block-sum, for a chain that starts (box clamp) at row s0.
 * C must hold the previous row's C (or P2 at y == s0). Mirrors getRawMatchingCost and the
 * pass-1 block of computeDisparitySGBM.  Cprev may alias C. */
static void cost_row(cost_state* cs, const uint8_t* L, const uint8_t* R, size_t step, int width,
                     int height, const eff_params* e, int y, int s0, cost_t* C, const cost_t* Cprev)
{
    const int W1 = e->width1, D = e->D, SH2 = e->SH2;
    const size_t row = (size_t)W1 * D;
    int dy1 = y == s0 ? s0 : y + SH2, dy2 = y == s0 ? s0 + SH2 : dy1;
    for (int k = dy1; k <= dy2; k++) {
        cost_t* hsumAdd = cs->hsum + (size_t)(imin(k, height - 1) % cs->nrows) * row;
        if (k < height) {
            calc_pixel_cost_bt(L, R, step, width, height, k, e->minD, e->maxD, cs->pix,
                               cs->tab + TAB_OFS, cs->work, e->cn);
            hsum_row(cs->pix, hsumAdd, W1, D, e->SW2);
            if (y > s0) {
                const cost_t* hsumSub = cs->hsum + (size_t)(imax(y - SH2 - 1, s0) % cs->nrows) * row;
                for (size_t i = 0; i < row; i++) C[i] = (cost_t)(Cprev[i] + hsumAdd[i] - hsumSub[i]);
            }
        }
        if (y == s0) {
            int scale = k == s0 ? SH2 + 1 : 1;
            for (size_t i = 0; i < row; i++) C[i] = (cost_t)(C[i] + hsumAdd[i] * scale);
        }
    }
}

static int sgbm_rows(const uint8_t* L, const uint8_t* R, int width, int height, size_t step,
                     const orc_params* p, const eff_params* e, int16_t* disp, size_t dstride,
                     int16_t* cost_dump /* optional [H][W1][D] */)
{
    const int W1 = e->width1, D = e->D, P1 = e->P1, P2 = e->P2;
    const int fullDP = p->mode == ORC_MODE_HH;
    const int npasses = fullDP ? 2 : 1;
    const size_t row = (size_t)W1 * D;

    cost_t* Cbuf = (cost_t*)malloc(row * (fullDP ? height : 1) * sizeof(cost_t));
    cost_t* Sbuf = (cost_t*)calloc(row * (fullDP ? height : 1), sizeof(cost_t));
    int16_t* disp2 = (int16_t*)malloc((size_t)width * sizeof(int16_t));
    int* disp2cost = (int*)malloc((size_t)width * sizeof(int));
    lr_bufs lb;
    lb.W1 = W1; lb.D = D;
    lb.L = (cost_t*)malloc((size_t)2 * (W1 + 2) * NDIR * (D + 2) * sizeof(cost_t));
    lb.minL = (int*)malloc((size_t)2 * (W1 + 2) * NDIR * sizeof(int));
    cost_state cs;
    int rc = cost_state_init(&cs, e, width);
    if (!Cbuf || !Sbuf || !disp2 || !disp2cost || !lb.L || !lb.minL || rc) { rc = -1; goto done; }

    /* initCBuf(P2): "add P2 to every C(x,y); it saves a few operations in the inner loops" */
    for (size_t i = 0; i < row * (fullDP ? height : 1); i++) Cbuf[i] = (cost_t)P2;

    for (int pass = 1; pass <= npasses; pass++) {
        int y1, y2, dy, x1, x2, dx;
        if (pass == 1) { y1 = 0; y2 = height; dy = 1; x1 = 0; x2 = W1; dx = 1; }
        else { y1 = height - 1; y2 = -1; dy = -1; x1 = W1 - 1; x2 = -1; dx = -1; }
        int lrID = 0;
        lr_clear(&lb);

        for (int y = y1; y != y2; y += dy) {
            cost_t* C = fullDP ? Cbuf + (size_t)y * row : Cbuf;
            cost_t* S = fullDP ? Sbuf + (size_t)y * row : Sbuf;
            int16_t* drow = disp + (size_t)y * dstride;

            if (pass == 1) {
                const cost_t* Cprev = (!fullDP || y == 0) ? C : C - row;
                cost_row(&cs, L, R, step, width, height, e, y, 0, C, Cprev);
                if (cost_dump) memcpy(cost_dump + (size_t)y * row, C, row * sizeof(cost_t));
                memset(S, 0, row * sizeof(cost_t));
            }

            /* forward x pass: directions 0:(-dx,0) 1:(-1,-dy) 2:(0,-dy) 3:(+1,-dy) */
            for (int x = x1; x != x2; x += dx) {
                const cost_t* Cp = C + (size_t)x * D;
                cost_t* Sp = S + (size_t)x * D;
                const cost_t* Lp0 = lr_at(&lb, lrID, x - dx, 0);
                const cost_t* Lp1 = lr_at(&lb, 1 - lrID, x - 1, 1);
                const cost_t* Lp2 = lr_at(&lb, 1 - lrID, x, 2);
                const cost_t* Lp3 = lr_at(&lb, 1 - lrID, x + 1, 3);
                int m0 = *minl_at(&lb, lrID, x - dx, 0);
                int m1 = *minl_at(&lb, 1 - lrID, x - 1, 1);
                int m2 = *minl_at(&lb, 1 - lrID, x, 2);
                int m3 = *minl_at(&lb, 1 - lrID, x + 1, 3);
                cost_t* Lo0 = lr_at(&lb, lrID, x, 0);
                cost_t* Lo1 = lr_at(&lb, lrID, x, 1);
                cost_t* Lo2 = lr_at(&lb, lrID, x, 2);
                cost_t* Lo3 = lr_at(&lb, lrID, x, 3);
                *minl_at(&lb, lrID, x, 0) = path_step(Cp, Lp0, m0, Lo0, D, P1, P2);
                *minl_at(&lb, lrID, x, 1) = path_step(Cp, Lp1, m1, Lo1, D, P1, P2);
                *minl_at(&lb, lrID, x, 2) = path_step(Cp, Lp2, m2, Lo2, D, P1, P2);
                *minl_at(&lb, lrID, x, 3) = path_step(Cp, Lp3, m3, Lo3, D, P1, P2);
                for (int d = 0; d < D; d++)
                    Sp[d] = sat16(Sp[d] + Lo0[d] + Lo1[d] + Lo2[d] + Lo3[d]);
            }

            if (pass == npasses) {
                for (int x = 0; x < width; x++) {
                    drow[x] = (int16_t)e->invalid_scaled;
                    disp2[x] = (int16_t)e->invalid_scaled;
                    disp2cost[x] = MAX_COST;
                }
                for (int x = W1 - 1; x >= 0; x--) {
                    cost_t* Sp = S + (size_t)x * D;
                    if (npasses == 1) {
                        /* direction 4: (+1, 0), accumulated in the WTA loop (x descending) */
                        const cost_t* Lp0 = lr_at(&lb, lrID, x + 1, 0);
                        int m0 = *minl_at(&lb, lrID, x + 1, 0);
                        cost_t* Lo0 = lr_at(&lb, lrID, x, 0);
                        *minl_at(&lb, lrID, x, 0) = path_step(C + (size_t)x * D, Lp0, m0, Lo0, D, P1, P2);
                        for (int d = 0; d < D; d++) Sp[d] = sat16(Sp[d] + Lo0[d]);
                    }
                    int minS, best, d16;
                    if (!wta_pixel(Sp, e, &minS, &best, &d16)) continue;
                    int _x2 = x + e->minX1 - best - e->minD;
                    /* best == -1 (every S saturated) can put _x2 one past the row: OpenCV reads */
                    /* out of range there, but its cost MAX_COST never replaces disp2cost       */
                    if (_x2 >= 0 && _x2 < width && disp2cost[_x2] > minS) {
                        disp2cost[_x2] = minS;
                        disp2[_x2] = (int16_t)(best + e->minD);
                    }
                    drow[x + e->minX1] = (int16_t)d16;
                }
                lr_check_row(drow, disp2, width, e);
            }
            lrID = 1 - lrID;
        }
    }
    rc = 0;
done:
    cost_state_free(&cs);
    free(Cbuf); free(Sbuf); free(disp2); free(disp2cost); free(lb.L); free(lb.minL);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* MODE_HH4: computeDisparitySGBM_HH4 (OpenCV 4.x).  4 paths over a full-DP cost buffer:        */
/*   CalcVerticalSums   -- per column, pass 1 top-to-bottom (C rows formed as in MODE_HH, so the */
/*                         bottom rows the running sum never reaches keep P2; S cleared), pass 2 */
/*                         bottom-to-top; each adds its L into S (saturating);                   */
/*   CalcHorizontalSums -- per row, left-to-right, then right-to-left with the WTA (scalar       */
/*                         uniqueness, x descending for disp2), then the row's LR check.         */
/* ------------------------------------------------------------------------------------------ */
static int sgbm_hh4(const uint8_t* L, const uint8_t* R, int width, int height, size_t step,
                    const eff_params* e, int16_t* disp, size_t dstride)
{
    const int W1 = e->width1, D = e->D, P1 = e->P1, P2 = e->P2;
    const size_t row = (size_t)W1 * D;
    const size_t lst = (size_t)D + 2; /* L record with the d = -1 / d = D sentinels */
    cost_t* Cbuf = (cost_t*)malloc(row * height * sizeof(cost_t));
    cost_t* Sbuf = (cost_t*)calloc(row * height, sizeof(cost_t));
    cost_t* Lv = (cost_t*)malloc(2 * (size_t)W1 * lst * sizeof(cost_t)); /* [2][W1][D+2] */
    int* mv = (int*)malloc(2 * (size_t)W1 * sizeof(int));
    cost_t* Lh = (cost_t*)malloc(2 * lst * sizeof(cost_t));
    int16_t* disp2 = (int16_t*)malloc((size_t)width * sizeof(int16_t));
    int* disp2cost = (int*)malloc((size_t)width * sizeof(int));
    cost_state cs;
    int rc = cost_state_init(&cs, e, width);
    if (!Cbuf || !Sbuf || !Lv || !mv || !Lh || !disp2 || !disp2cost || rc) { rc = -1; goto done; }
    for (size_t i = 0; i < row * height; i++) Cbuf[i] = (cost_t)P2;

    /* CalcVerticalSums */
    for (int pass = 1; pass <= 2; pass++) {
        for (size_t i = 0; i < 2 * (size_t)W1; i++) {
            cost_t* l = Lv + i * lst;
            for (size_t d = 0; d < lst; d++) l[d] = 0;
            l[0] = l[D + 1] = MAX_COST;
            mv[i] = 0;
        }
        int cur = 0;
        for (int k = 0; k < height; k++) {
            const int y = pass == 1 ? k : height - 1 - k;
            cost_t* C = Cbuf + (size_t)y * row;
            cost_t* S = Sbuf + (size_t)y * row;
            if (pass == 1) cost_row(&cs, L, R, step, width, height, e, y, 0, C, y == 0 ? C : C - row);
            for (int x = 0; x < W1; x++) {
                const cost_t* Lp = Lv + ((size_t)(1 - cur) * W1 + x) * lst + 1;
                cost_t* Lo = Lv + ((size_t)cur * W1 + x) * lst + 1;
                mv[cur * W1 + x] = path_step(C + (size_t)x * D, Lp, mv[(1 - cur) * W1 + x], Lo, D, P1, P2);
                cost_t* Sp = S + (size_t)x * D;
                for (int d = 0; d < D; d++) Sp[d] = sat16(Sp[d] + Lo[d]);
            }
            cur = 1 - cur;
        }
    }

    /* CalcHorizontalSums */
    for (int y = 0; y < height; y++) {
        const cost_t* C = Cbuf + (size_t)y * row;
        cost_t* S = Sbuf + (size_t)y * row;
        int16_t* drow = disp + (size_t)y * dstride;
        for (int x = 0; x < width; x++) {
            drow[x] = (int16_t)e->invalid_scaled;
            disp2[x] = (int16_t)e->invalid_scaled;
            disp2cost[x] = MAX_COST;
        }
        for (int dir = 0; dir < 2; dir++) {
            for (size_t i = 0; i < 2; i++) {
                cost_t* l = Lh + i * lst;
                for (size_t d = 0; d < lst; d++) l[d] = 0;
                l[0] = l[D + 1] = MAX_COST;
            }
            int m = 0, cur = 0;
            for (int k = 0; k < W1; k++) {
                const int x = dir == 0 ? k : W1 - 1 - k;
                cost_t* Lo = Lh + (size_t)cur * lst + 1;
                m = path_step(C + (size_t)x * D, Lh + (size_t)(1 - cur) * lst + 1, m, Lo, D, P1, P2);
                cur = 1 - cur;
                cost_t* Sp = S + (size_t)x * D;
                for (int d = 0; d < D; d++) Sp[d] = sat16(Sp[d] + Lo[d]);
                if (dir == 0) continue;
                int minS, best, d16;
                if (!wta_pixel(Sp, e, &minS, &best, &d16)) continue;
                int _x2 = x + e->minX1 - best - e->minD;
                if (_x2 >= 0 && _x2 < width && disp2cost[_x2] > minS) {
                    disp2cost[_x2] = minS;
                    disp2[_x2] = (int16_t)(best + e->minD);
                }
                drow[x + e->minX1] = (int16_t)d16;
            }
        }
        lr_check_row(drow, disp2, width, e);
    }
    rc = 0;
done:
    cost_state_free(&cs);
    free(Cbuf); free(Sbuf); free(Lv); free(mv); free(Lh); free(disp2); free(disp2cost);
    return rc;
}

/* ------------------------------------------------------------------------------------------ */
/* A.7: computeDisparity3WaySGBM.  OpenCV 4.x fixes nstripes = 4 ("the number of stripes is    */
/* fixed, disregarding the number of threads/processors, to make the results fully              */
/* reproducible"); stripe_overlap = (SADWindowSize/2 + 1) + ceil(0.1 * stripe_sz).  Each stripe */
/* restarts the vertical path and the vertical box sum at its first (overlap) row.              */
/* ------------------------------------------------------------------------------------------ */
static int sgbm3way_stripe(const uint8_t* L, const uint8_t* R, int width, int height, size_t step,
                           const eff_params* e, int src_start, int src_end, int out_start,
                           int16_t* disp, size_t dstride)
{
    const int W1 = e->width1, D = e->D, P1 = e->P1, P2 = e->P2;
    const size_t row = (size_t)W1 * D;
    cost_t* C = (cost_t*)malloc(row * sizeof(cost_t));
    cost_t* hor = (cost_t*)calloc((size_t)(W1 + 1) * (D + 2), sizeof(cost_t)); /* left path, x=-1 pad */
    cost_t* ver = (cost_t*)calloc((size_t)W1 * (D + 2), sizeof(cost_t));       /* top path state     */
    int* verMin = (int*)calloc((size_t)W1, sizeof(int));
    cost_t* right = (cost_t*)calloc((size_t)2 * (D + 2), sizeof(cost_t));
    cost_t* Ssum = (cost_t*)calloc(row, sizeof(cost_t));
    int* horMin = (int*)calloc((size_t)W1 + 1, sizeof(int));
    int16_t* disp2 = (int16_t*)malloc((size_t)width * sizeof(int16_t));
    int* disp2cost = (int*)malloc((size_t)width * sizeof(int));
    cost_state cs;
    int rc = cost_state_init(&cs, e, width);
    if (!C || !hor || !ver || !verMin || !right || !Ssum || !horMin || !disp2 || !disp2cost || rc) {
        rc = -1; goto done;
    }
#define HOR(x) (hor + (size_t)((x) + 1) * (D + 2) + 1)
#define VER(x) (ver + (size_t)(x) * (D + 2) + 1)
    for (int x = -1; x < W1; x++) { HOR(x)[-1] = HOR(x)[D] = MAX_COST; }
    for (int x = 0; x < W1; x++) { VER(x)[-1] = VER(x)[D] = MAX_COST; }
    for (size_t i = 0; i < row; i++) C[i] = (cost_t)P2; /* curCostVolumeLine initialised to P2 */

    for (int y = src_start; y < src_end; y++) {
        cost_row(&cs, L, R, step, width, height, e, y, src_start, C, C);
        int16_t* drow = y >= out_start ? disp + (size_t)y * dstride : NULL;

        for (int x = 0; x < width; x++) {
            disp2[x] = (int16_t)e->invalid_scaled;
            disp2cost[x] = MAX_COST;
        }
        /* forward pass: left-to-right path and top-to-bottom path */
        for (int x = 0; x < W1; x++) {
            const cost_t* Cp = C + (size_t)x * D;
            horMin[x + 1] = path_step(Cp, HOR(x - 1), horMin[x], HOR(x), D, P1, P2);
            cost_t tmp[1024 + 2];
            cost_t* Lv = tmp + 1;
            verMin[x] = path_step(Cp, VER(x), verMin[x], Lv, D, P1, P2);
            memcpy(VER(x), Lv, (size_t)D * sizeof(cost_t));
        }
        /* backward pass: right-to-left path, total cost, WTA */
        cost_t* Rp = right + 1;          /* previous pixel's right-path state */
        cost_t* Rn = right + (D + 2) + 1;
        for (int d = -1; d <= D; d++) { Rp[d] = 0; Rn[d] = 0; }
        Rp[-1] = Rp[D] = Rn[-1] = Rn[D] = MAX_COST;
        int rmin = 0;
        for (int x = W1 - 1; x >= 0; x--) {
            const cost_t* Cp = C + (size_t)x * D;
            rmin = path_step(Cp, Rp, rmin, Rn, D, P1, P2);
            cost_t* Sp = Ssum + (size_t)x * D;
            for (int d = 0; d < D; d++) Sp[d] = sat16((int)HOR(x)[d] + Rn[d] + VER(x)[d]);
            cost_t* t = Rp; Rp = Rn; Rn = t;
            if (!drow) continue;
            int minS, best, d16;
            if (!wta_pixel(Sp, e, &minS, &best, &d16)) continue;
            int _x2 = x + e->minX1 - best - e->minD;
            if (_x2 >= 0 && _x2 < width && disp2cost[_x2] > minS) {
                disp2cost[_x2] = minS;
                disp2[_x2] = (int16_t)(best + e->minD);
            }
            drow[x + e->minX1] = (int16_t)d16;
        }
        if (drow) lr_check_row(drow, disp2, width, e);
    }
#undef HOR
#undef VER
    rc = 0;
done:
    cost_state_free(&cs);
    free(C); free(hor); free(ver); free(verMin); free(right); free(Ssum); free(horMin);
    free(disp2); free(disp2cost);
    return rc;
}

static int sgbm3way(const uint8_t* L, const uint8_t* R, int width, int height, size_t step,
                    const orc_params* p, const eff_params* e, int16_t* disp, size_t dstride)
{
    if (e->D > 1024) return -2;
    const int nstripes = p->nstripes > 0 ? p->nstripes : 4;
    const int stripe_sz = (int)ceil(height / (double)nstripes);
    const int stripe_overlap = (p->blockSize / 2 + 1) + (int)ceil(0.1 * stripe_sz);
    for (int y = 0; y < height; y++)
        for (int x = 0; x < width; x++) disp[(size_t)y * dstride + x] = (int16_t)e->invalid_scaled;
    for (int s = 0; s < nstripes; s++) {
        int src_start = imax(imin(s * stripe_sz - stripe_overlap, height), 0);
        int src_end = imin((s + 1) * stripe_sz, height);
        int out_start = s * stripe_sz;
        if (out_start >= height) break;
        int rc = sgbm3way_stripe(L, R, width, height, step, e, src_start, src_end, out_start, disp, dstride);
        if (rc) return rc;
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
int orc_sgbm_compute_cn(const uint8_t* left, const uint8_t* right, int width, int height,
                        size_t stride, int cn, const orc_params* p, int16_t* disp,
                        size_t disp_stride, int stages)
{
    eff_params e;
    if (!left || !right || !disp || !p || width <= 0 || height <= 0) return -1;
    if (cn != 1 && cn != 3) return -1;
    int rc = make_eff(p, width, &e);
    if (rc) return rc;
    e.cn = cn;
    if (p->mode != ORC_MODE_SGBM && p->mode != ORC_MODE_HH && p->mode != ORC_MODE_SGBM_3WAY &&
        p->mode != ORC_MODE_HH4)
        return -3;
    int16_t* raw = (int16_t*)malloc((size_t)width * height * sizeof(int16_t));
    if (!raw) return -1;
    if (e.width1 <= 0) {
        for (size_t i = 0; i < (size_t)width * height; i++) raw[i] = (int16_t)e.invalid_scaled;
    } else if (e.width1 <= e.SW2) {
        free(raw);
        return -4; /* OpenCV reads pixDiff[SW2*Da] out of range here */
    } else if (p->mode == ORC_MODE_SGBM_3WAY) {
        rc = sgbm3way(left, right, width, height, stride, p, &e, raw, (size_t)width);
    } else if (p->mode == ORC_MODE_HH4) {
        rc = sgbm_hh4(left, right, width, height, stride, &e, raw, (size_t)width);
    } else {
        rc = sgbm_rows(left, right, width, height, stride, p, &e, raw, (size_t)width, NULL);
    }
    if (rc) { free(raw); return rc; }
    if (stages & ORC_STAGE_MEDIAN) {
        int16_t* med = (int16_t*)malloc((size_t)width * height * sizeof(int16_t));
        orc_median3x3_s16(raw, med, width, height);
        memcpy(raw, med, (size_t)width * height * sizeof(int16_t));
        free(med);
    }
    if ((stages & ORC_STAGE_SPECKLE) && p->speckleWindowSize > 0)
        orc_filter_speckles_s16(raw, width, height, e.invalid_scaled, p->speckleWindowSize,
                                DISP_SCALE * p->speckleRange);
    for (int y = 0; y < height; y++)
        memcpy(disp + (size_t)y * disp_stride, raw + (size_t)y * width, (size_t)width * sizeof(int16_t));
    free(raw);
    return 0;
}

int orc_sgbm_compute_stages(const uint8_t* left, const uint8_t* right, int width, int height,
                            size_t stride, const orc_params* p, int16_t* disp,
                            size_t disp_stride, int stages)
{
    return orc_sgbm_compute_cn(left, right, width, height, stride, 1, p, disp, disp_stride, stages);
}

int orc_sgbm_compute(const uint8_t* left, const uint8_t* right, int width, int height,
                     size_t stride, const orc_params* p, int16_t* disp, size_t disp_stride)
{
    return orc_sgbm_compute_stages(left, right, width, height, stride, p, disp, disp_stride,
                                   ORC_STAGE_MEDIAN | ORC_STAGE_SPECKLE);
}

int orc_cost_volume_cn(const uint8_t* left, const uint8_t* right, int width, int height,
                       size_t stride, int cn, const orc_params* p, int16_t* out)
{
    eff_params e;
    if (cn != 1 && cn != 3) return -1;
    int rc = make_eff(p, width, &e);
    if (rc) return rc;
    e.cn = cn;
    if (e.width1 <= e.SW2) return -4;
    const size_t row = (size_t)e.width1 * e.D;
    cost_state cs;
    if (cost_state_init(&cs, &e, width)) return -1;
    const int fullDP = p->mode == ORC_MODE_HH || p->mode == ORC_MODE_HH4;
    cost_t* C = (cost_t*)malloc(row * sizeof(cost_t));
    for (size_t i = 0; i < row; i++) C[i] = (cost_t)e.P2;
    for (int y = 0; y < height; y++) {
        if (fullDP && y > 0) {
            /* full-DP buffers start every row at P2 and update it from the previous row */
            cost_t* Cy = out + (size_t)y * row;
            for (size_t i = 0; i < row; i++) Cy[i] = (cost_t)e.P2;
            cost_row(&cs, left, right, stride, width, height, &e, y, 0, Cy, out + (size_t)(y - 1) * row);
        } else {
            cost_row(&cs, left, right, stride, width, height, &e, y, 0, C, C);
            memcpy(out + (size_t)y * row, C, row * sizeof(cost_t));
        }
    }
    free(C);
    cost_state_free(&cs);
    return 0;
}

int orc_cost_volume(const uint8_t* left, const uint8_t* right, int width, int height,
                    size_t stride, const orc_params* p, int16_t* out)
{
    return orc_cost_volume_cn(left, right, width, height, stride, 1, p, out);
}

int orc_pixel_cost_row(const uint8_t* left, const uint8_t* right, int width, int height,
                       size_t stride, int y, int minD, int numD, int preFilterCap, int16_t* out)
{
    uint8_t tab[TAB_OFS * 2 + 256];
    int maxD = minD + numD;
    if (imax(maxD, 0) >= width + imin(minD, 0)) return -4;
    uint8_t* work = (uint8_t*)malloc((size_t)width * 6);
    make_clip_tab(imax(preFilterCap, 15) | 1, tab);
    calc_pixel_cost_bt(left, right, stride, width, height, y, minD, maxD, out, tab + TAB_OFS, work, 1);
    free(work);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* A.10 medianBlur 3x3 (replicate border).                                                     */
/* ------------------------------------------------------------------------------------------ */
static int cmp16(const void* a, const void* b)
{
    return (int)*(const int16_t*)a - (int)*(const int16_t*)b;
}

void orc_median3x3_s16(const int16_t* src, int16_t* dst, int width, int height)
{
    for (int y = 0; y < height; y++) {
        for (int x = 0; x < width; x++) {
            int16_t v[9];
            int k = 0;
            for (int dy = -1; dy <= 1; dy++) {
                int yy = imin(imax(y + dy, 0), height - 1);
                for (int dx = -1; dx <= 1; dx++) {
                    int xx = imin(imax(x + dx, 0), width - 1);
                    v[k++] = src[(size_t)yy * width + xx];
                }
            }
            qsort(v, 9, sizeof(int16_t), cmp16);
            dst[(size_t)y * width + x] = v[4];
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* A.11 filterSpeckles: 4-connected flood fill (LIFO wavefront), regions whose pixel count is   */
/* <= maxSpeckleSize are set to newVal.                                                        */
/* ------------------------------------------------------------------------------------------ */
void orc_filter_speckles_s16(int16_t* img, int width, int height, int newVal,
                             int maxSpeckleSize, int maxDiff)
{
    const int npixels = width * height;
    int* labels = (int*)calloc((size_t)npixels, sizeof(int));
    int* wbuf = (int*)malloc((size_t)npixels * 2 * sizeof(int));
    uint8_t* rtype = (uint8_t*)calloc((size_t)npixels + 1, 1);
    int curlabel = 0;
    for (int i = 0; i < height; i++) {
        int16_t* ds = img + (size_t)i * width;
        int* ls = labels + (size_t)i * width;
        for (int j = 0; j < width; j++) {
            if (ds[j] == newVal) continue;
            if (ls[j]) {
                if (rtype[ls[j]]) ds[j] = (int16_t)newVal;
                continue;
            }
            int nw = 0;
            int px = j, py = i;
            curlabel++;
            int count = 0;
            ls[j] = curlabel;
            for (;;) {
                count++;
                int16_t* dpp = img + (size_t)py * width + px;
                int dp = *dpp;
                int* lpp = labels + (size_t)py * width + px;
                if (py < height - 1 && !lpp[width] && dpp[width] != newVal && abs(dp - dpp[width]) <= maxDiff) {
                    lpp[width] = curlabel; wbuf[2 * nw] = px; wbuf[2 * nw + 1] = py + 1; nw++;
                }
                if (py > 0 && !lpp[-width] && dpp[-width] != newVal && abs(dp - dpp[-width]) <= maxDiff) {
                    lpp[-width] = curlabel; wbuf[2 * nw] = px; wbuf[2 * nw + 1] = py - 1; nw++;
                }
                if (px < width - 1 && !lpp[1] && dpp[1] != newVal && abs(dp - dpp[1]) <= maxDiff) {
                    lpp[1] = curlabel; wbuf[2 * nw] = px + 1; wbuf[2 * nw + 1] = py; nw++;
                }
                if (px > 0 && !lpp[-1] && dpp[-1] != newVal && abs(dp - dpp[-1]) <= maxDiff) {
                    lpp[-1] = curlabel; wbuf[2 * nw] = px - 1; wbuf[2 * nw + 1] = py; nw++;
                }
                if (nw == 0) break;
                nw--;
                px = wbuf[2 * nw]; py = wbuf[2 * nw + 1];
            }
            if (count <= maxSpeckleSize) {
                rtype[ls[j]] = 1;
                ds[j] = (int16_t)newVal;
            } else {
                rtype[ls[j]] = 0;
            }
        }
    }
    free(labels); free(wbuf); free(rtype);
}

/* ------------------------------------------------------------------------------------------ */
/* A.12 reprojectImageTo3D: homg = Matx44d(Q) * Vec4d(x, y, d, 1) (sequential sums from 0),     */
/* Vec3f(homg[0..2]) then /= homg[3] as multiplication by (1.0 / homg[3]) in double, rounded to */
/* float; handleMissingValues sets Z = 10000 where |d - min(disp)| <= FLT_EPSILON.              */
/* ------------------------------------------------------------------------------------------ */
void orc_reproject_f32(const float* disp, int width, int height, const double Q[16],
                       int handle_missing, float* xyz)
{
    double minDisparity = FLT_MAX;
    if (handle_missing) {
        for (size_t i = 0; i < (size_t)width * height; i++)
            if (disp[i] < minDisparity) minDisparity = disp[i];
    }
    for (int y = 0; y < height; y++) {
        for (int x = 0; x < width; x++) {
            double d = disp[(size_t)y * width + x];
            double v[4] = {(double)x, (double)y, d, 1.0};
            double h[4];
            for (int i = 0; i < 4; i++) {
                double s = 0;
                for (int k = 0; k < 4; k++) s += Q[i * 4 + k] * v[k];
                h[i] = s;
            }
            double ia = 1. / h[3];
            float* o = xyz + ((size_t)y * width + x) * 3;
            for (int i = 0; i < 3; i++) {
                /* volatile: GCC 11's SLP vectoriser drops this float narrowing at -O3 */
                volatile float f = (float)h[i];
                o[i] = (float)((double)f * ia);
            }
            if (fabs(d - minDisparity) <= FLT_EPSILON) o[2] = 10000.f;
        }
    }
}

/* A.13 pre-steps ---------------------------------------------------------------------------- */
void orc_bgr2gray(const uint8_t* bgr, int width, int height, size_t bgr_stride, uint8_t* gray)
{
    for (int y = 0; y < height; y++) {
        const uint8_t* s = bgr + (size_t)y * bgr_stride;
        for (int x = 0; x < width; x++) {
            int b = s[3 * x], g = s[3 * x + 1], r = s[3 * x + 2];
            gray[(size_t)y * width + x] = (uint8_t)((b * 1868 + g * 9617 + r * 4899 + (1 << 13)) >> 14);
        }
    }
}

void orc_resize_area_half(const uint8_t* src, int width, int height, size_t stride, uint8_t* dst)
{
    int dw = width / 2, dh = height / 2;
    for (int y = 0; y < dh; y++) {
        const uint8_t* a = src + (size_t)(2 * y) * stride;
        const uint8_t* b = a + stride;
        for (int x = 0; x < dw; x++)
            dst[(size_t)y * dw + x] = (uint8_t)((a[2 * x] + a[2 * x + 1] + b[2 * x] + b[2 * x + 1] + 2) >> 2);
    }
}

void orc_disp_to_float(const int16_t* disp, int n, float* out)
{
    for (int i = 0; i < n; i++) out[i] = (float)disp[i] * 0.0625f;
}

/*
 * wls_oracle.c -- CPU restatement of ximgproc's DisparityWLSFilter + FastGlobalSmootherFilter.
 * TEST INFRASTRUCTURE ONLY; see wls_oracle.h for what is restated and why parity is unpinned.
 * Built with -ffp-contract=off (oracle/Makefile): every float operation below is rounded on its
 * own, the order the GPU kernels (sdr_wls.hip) reproduce.
 */
#include "wls_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define FGS_LEVELS 65026 /* 255^2 + 1: squared difference of two 8-bit gray levels */

void orc_wls_params_for_sgbm(int minDisparity, int numDisparities, int blockSize, int width,
                             int height, orc_wls_params* p) {
    /* createDisparityWLSFilter(Ptr<StereoSGBM>): offsets (max(0,min+num), max(0,-min), 0, 0),
     * depth-discontinuity radius ceil(0.5*wsize); DisparityWLSFilterImpl::init defaults. */
    const int l = minDisparity + numDisparities > 0 ? minDisparity + numDisparities : 0;
    const int r = -minDisparity > 0 ? -minDisparity : 0;
    p->lambda = 8000.0;
    p->sigma_color = 1.5;
    p->lrc_thresh = 24;
    p->depth_disc_radius = (int)ceil(0.5 * blockSize);
    p->roll_off = 0.001f;
    p->lambda_attenuation = 0.25;
    p->num_iter = 3;
    p->roi_x = l;
    p->roi_y = 0;
    p->roi_w = width - l - r;
    p->roi_h = height;
    p->min_disp = minDisparity;
    p->fgs_solver = ORC_FGS_THOMAS;
}

void orc_fgs_lut(double sigma_color, float* lut) {
    const float s = (float)sigma_color;
    for (int i = 0; i < FGS_LEVELS; i++) lut[i] = -expf(-sqrtf((float)i) / s);
}

/* cv::borderInterpolate(p, len, BORDER_REFLECT_101) */
static int reflect101(int p, int len) {
    if (len == 1) return 0;
    while (p < 0 || p >= len) {
        if (p < 0) p = -p;
        else p = 2 * len - 2 - p;
    }
    return p;
}

void orc_wls_disc_map(const int16_t* d, int W, int H, int rx, int ry, int rw, int rh, int radius,
                      float roll_off, float* out) {
    for (int i = 0; i < W * H; i++) out[i] = 1.0f;
    if (rw <= 0 || rh <= 0) return;
    const int k = 2 * radius + 1;
    const double scale = 1.0 / (double)(k * k);
    for (int i = 0; i < rh; i++) {
        for (int j = 0; j < rw; j++) {
            long long s = 0, s2 = 0;
            for (int a = -radius; a <= radius; a++) {
                const int ii = reflect101(i + a, rh);
                for (int b = -radius; b <= radius; b++) {
                    const int jj = reflect101(j + b, rw);
                    const long long v = d[(size_t)(ry + ii) * W + rx + jj];
                    s += v;
                    s2 += v * v;
                }
            }
            /* boxFilter(CV_32F) and sqrBoxFilter(CV_32F): (float)(sum * scale) */
            const float mean = (float)((double)s * scale);
            const float msq = (float)((double)s2 * scale);
            const float var = msq - mean * mean;
            const float c = 1.0f - roll_off * var;
            out[(size_t)(ry + i) * W + rx + j] = c > 0.0f ? c : 0.0f;
        }
    }
}

void orc_wls_confidence(const int16_t* dl, const int16_t* dr, int W, int H, const orc_wls_params* p,
                        float* conf) {
    float* rd = (float*)malloc(sizeof(float) * (size_t)W * H);
    /* right view ROI mirrors the left one (computeConfidenceMap) */
    const int rrx = W - (p->roi_x + p->roi_w), rry = p->roi_y, rrw = p->roi_w, rrh = p->roi_h;
    orc_wls_disc_map(dl, W, H, p->roi_x, p->roi_y, p->roi_w, p->roi_h, p->depth_disc_radius,
                     p->roll_off, conf);
    orc_wls_disc_map(dr, W, H, rrx, rry, rrw, rrh, p->depth_disc_radius, p->roll_off, rd);
    /* ComputeDiscontinuityAwareLRC: rows and columns of the left ROI (stripes over its height) */
    for (int i = p->roi_y; i < p->roi_y + p->roi_h; i++) {
        const int16_t* L = dl + (size_t)i * W;
        const int16_t* R = dr + (size_t)i * W;
        float* c = conf + (size_t)i * W;
        const float* rc = rd + (size_t)i * W;
        for (int j = p->roi_x; j < p->roi_x + p->roi_w; j++) {
            const int ridx = j - (L[j] >> 4);
            if (ridx >= rrx && ridx < rrx + rrw) {
                if (abs((int)L[j] + (int)R[ridx]) < p->lrc_thresh) c[j] = c[j] < rc[ridx] ? c[j] : rc[ridx];
                else c[j] = 0.0f;
            }
        }
    }
    for (size_t i = 0; i < (size_t)W * H; i++) conf[i] = 255.0f * conf[i];
    free(rd);
}

/* one tridiagonal solve along a line of n samples with stride s:
 *   (1 - lam*(C[k-1] + C[k])) u_k + lam*C[k-1] u_{k-1} + lam*C[k] u_{k+1} = f_k,  C = -w <= 0 */
static void fgs_line(float* u, const float* C, float* t, int n, size_t s, float lam) {
    float denom = 1.0f - lam * C[0];
    t[0] = lam * C[0] / denom;
    u[0] = u[0] / denom;
    for (int k = 1; k < n; k++) {
        const float a = lam * C[(size_t)(k - 1) * s];
        const float c = lam * C[(size_t)k * s];
        denom = 1.0f - c - a * (1.0f + t[(size_t)(k - 1) * s]);
        t[(size_t)k * s] = c / denom;
        u[(size_t)k * s] = (u[(size_t)k * s] - a * u[(size_t)(k - 1) * s]) / denom;
    }
    for (int k = n - 2; k >= 0; k--) u[(size_t)k * s] = u[(size_t)k * s] - t[(size_t)k * s] * u[(size_t)(k + 1) * s];
}

/* The same system solved by parallel cyclic reduction (the engine's k_fgs_pcr follows this
 * operation order exactly).  Equation k of a line: a_k u_{k-1} + b_k u_k + c_k u_{k+1} = d_k with
 *   c_k = lam*C[k] <= 0,  a_k = lam*C[k-1] <= 0 (0 at k = 0),  row sum e_k = a_k + b_k + c_k = 1.
 * Stage s (s = 1, 2, 4, ... < n) eliminates u_{k-s} and u_{k+s} from every equation at once,
 * using the neighbours' reciprocal diagonals r = 1/b (zeros stand for a missing neighbour):
 *   k1 = a_k r_{k-s} <= 0;  k2 = c_k r_{k+s} <= 0
 *   a_k' = -(a_{k-s} k1);  c_k' = -(c_{k+s} k2);  e_k' = (e_k - e_{k-s} k1) - e_{k+s} k2
 *   b_k' = (e_k' - a_k') - c_k';   d_k' = (d_k - d_{k-s} k1) - d_{k+s} k2
 * after which every equation is decoupled: u_k = d_k / b_k.  The diagonal is carried as the row
 * sum (the system is an M-matrix: every term of e' and b' is non-negative), never as
 * b - c k1 - a k2, whose terms cancel to about 1/(4 lam) of their size at lam = 8000 and would
 * lose ~14 bits per stage.  `w` holds 11 floats per sample. */
static void fgs_line_pcr(float* u, const float* C, float* w, int n, size_t s, float lam) {
    float *a = w, *e = w + n, *c = w + 2 * n, *d = w + 3 * n, *r = w + 4 * n, *b = w + 5 * n;
    float *a2 = w + 6 * n, *e2 = w + 7 * n, *c2 = w + 8 * n, *d2 = w + 9 * n, *b2 = w + 10 * n;
    for (int k = 0; k < n; k++) {
        c[k] = lam * C[(size_t)k * s];
        a[k] = k > 0 ? lam * C[(size_t)(k - 1) * s] : 0.0f;
        e[k] = 1.0f;
        b[k] = (1.0f - a[k]) - c[k];
        d[k] = u[(size_t)k * s];
    }
    for (int st = 1; st < n; st *= 2) {
        for (int k = 0; k < n; k++) r[k] = 1.0f / b[k];
        for (int k = 0; k < n; k++) {
            const int m = k - st, q = k + st;
            const float am = m >= 0 ? a[m] : 0.0f, em = m >= 0 ? e[m] : 0.0f;
            const float dm = m >= 0 ? d[m] : 0.0f, rm = m >= 0 ? r[m] : 0.0f;
            const float cp = q < n ? c[q] : 0.0f, ep = q < n ? e[q] : 0.0f;
            const float dp = q < n ? d[q] : 0.0f, rp = q < n ? r[q] : 0.0f;
            const float k1 = a[k] * rm;
            const float k2 = c[k] * rp;
            a2[k] = -(am * k1);
            c2[k] = -(cp * k2);
            e2[k] = (e[k] - em * k1) - ep * k2;
            b2[k] = (e2[k] - a2[k]) - c2[k];
            d2[k] = (d[k] - dm * k1) - dp * k2;
        }
        float* t;
        t = a; a = a2; a2 = t;
        t = e; e = e2; e2 = t;
        t = c; c = c2; c2 = t;
        t = d; d = d2; d2 = t;
        t = b; b = b2; b2 = t;
    }
    for (int k = 0; k < n; k++) u[(size_t)k * s] = d[k] / b[k];
}

void orc_fgs_filter_f32_ex(const uint8_t* g, size_t gs, int w, int h, double lambda,
                           double sigma, double att, int iters, int solver, float* img) {
    float* lut = (float*)malloc(sizeof(float) * FGS_LEVELS);
    float* Ch = (float*)malloc(sizeof(float) * (size_t)w * h);
    float* Cv = (float*)malloc(sizeof(float) * (size_t)w * h);
    const int nmax = w > h ? w : h;
    float* t = (float*)malloc(sizeof(float) * ((size_t)w * h > (size_t)11 * nmax ? (size_t)w * h : (size_t)11 * nmax));
    orc_fgs_lut(sigma, lut);
    for (int i = 0; i < h; i++)
        for (int j = 0; j < w; j++) {
            const int v = g[(size_t)i * gs + j];
            int dh = j + 1 < w ? v - g[(size_t)i * gs + j + 1] : 0;
            int dv = i + 1 < h ? v - g[(size_t)(i + 1) * gs + j] : 0;
            Ch[(size_t)i * w + j] = j + 1 < w ? lut[dh * dh] : 0.0f;
            Cv[(size_t)i * w + j] = i + 1 < h ? lut[dv * dv] : 0.0f;
        }
    float lam = (float)lambda;
    for (int n = 0; n < iters; n++) {
        if (solver == ORC_FGS_THOMAS) {
            for (int i = 0; i < h; i++) fgs_line(img + (size_t)i * w, Ch + (size_t)i * w, t + (size_t)i * w, w, 1, lam);
            for (int j = 0; j < w; j++) fgs_line(img + j, Cv + j, t + j, h, (size_t)w, lam);
        } else {
            for (int i = 0; i < h; i++) fgs_line_pcr(img + (size_t)i * w, Ch + (size_t)i * w, t, w, 1, lam);
            for (int j = 0; j < w; j++) fgs_line_pcr(img + j, Cv + j, t, h, (size_t)w, lam);
        }
        lam = lam * (float)att;
    }
    free(lut);
    free(Ch);
    free(Cv);
    free(t);
}

void orc_fgs_filter_f32(const uint8_t* g, size_t gs, int w, int h, double lambda, double sigma,
                        double att, int iters, float* img) {
    orc_fgs_filter_f32_ex(g, gs, w, h, lambda, sigma, att, iters, ORC_FGS_THOMAS, img);
}

/* saturate_cast<short>(float) = saturate_cast<short>(cvRound(v)): round to nearest even; cvRound
 * is cvtss2si, whose out-of-range/NaN result is INT_MIN (-> -32768 after saturation) */
static int16_t sat_s16(float v) {
    if (!(fabsf(v) < 2147483648.0f)) return -32768;
    const long r = lrintf(v);
    return (int16_t)(r < -32768 ? -32768 : (r > 32767 ? 32767 : r));
}

void orc_wls_filter(const int16_t* dl, const int16_t* dr, const uint8_t* guide, size_t gs, int W,
                    int H, const orc_wls_params* p, int16_t* out, float* conf_out) {
    float* conf = (float*)malloc(sizeof(float) * (size_t)W * H);
    orc_wls_confidence(dl, dr, W, H, p, conf);
    if (conf_out) memcpy(conf_out, conf, sizeof(float) * (size_t)W * H);
    const int16_t fill = (int16_t)(16 * (p->min_disp - 1));
    for (size_t i = 0; i < (size_t)W * H; i++) out[i] = fill;
    const int rw = p->roi_w, rh = p->roi_h;
    if (rw > 0 && rh > 0) {
        float* dc = (float*)malloc(sizeof(float) * (size_t)rw * rh);
        float* cc = (float*)malloc(sizeof(float) * (size_t)rw * rh);
        for (int i = 0; i < rh; i++)
            for (int j = 0; j < rw; j++) {
                const size_t o = (size_t)(p->roi_y + i) * W + p->roi_x + j;
                cc[(size_t)i * rw + j] = conf[o];
                dc[(size_t)i * rw + j] = conf[o] * (float)dl[o];
            }
        const uint8_t* g = guide + (size_t)p->roi_y * gs + p->roi_x;
        orc_fgs_filter_f32_ex(g, gs, rw, rh, p->lambda, p->sigma_color, p->lambda_attenuation, p->num_iter,
                              p->fgs_solver, dc);
        orc_fgs_filter_f32_ex(g, gs, rw, rh, p->lambda, p->sigma_color, p->lambda_attenuation, p->num_iter,
                              p->fgs_solver, cc);
        for (int i = 0; i < rh; i++)
            for (int j = 0; j < rw; j++) {
                const float c = cc[(size_t)i * rw + j];
                const float v = c != 0.0f ? dc[(size_t)i * rw + j] / c : 0.0f;
                out[(size_t)(p->roi_y + i) * W + p->roi_x + j] = sat_s16(v);
            }
        free(dc);
        free(cc);
    }
    free(conf);
}

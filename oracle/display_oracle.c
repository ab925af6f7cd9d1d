/*
 * display_oracle.c -- CPU restatement of the reference's display outputs.
 * TEST INFRASTRUCTURE ONLY: the checker of stereo_depth_ruler_amd/csrc/sdr_display.hip.
 *
 *   show_disparityMap   reference stereo_vision/src/stereo_disparity.cpp:42-73
 *   show_depthMap       stereo_disparity.cpp:83-124 (range EMA state: function-static doubles)
 *   overlay             stereo_vision/src/stereo_displayer.cpp:164-173 (JET, 0.7 / 0.3)
 *   depth_coverage      stereo_displayer.cpp:105-118
 *
 * PARITY UNPINNED against OpenCV 4.6, which is absent here.  Recorded assumptions
 * about OpenCV internals [R]:
 *   - convertTo(CV_32F, a) / convertTo(CV_8U, a, b) evaluate v*a + b in float with the scale and
 *     shift rounded to float, as one fused multiply-add (the AVX2 dispatch of convertScale), then
 *     cvRound (round half to even) and saturate; a float that cvRound cannot represent (NaN,
 *     |v| >= 2^31) becomes INT_MIN, i.e. 0 after saturation;
 *   - cv::pow(x, 0.6) on CV_32F is the power rounded to float (OpenCV's own log32f/exp32f tables
 *     may differ in the last float bit, which the x255 conversion hides except at rounding ties);
 *   - addWeighted on 8U evaluates fma(a, alpha, b*beta) + gamma in float, then cvRound/saturate;
 *   - minMaxLoc with a mask that selects nothing reports 0/0 (either way the reference falls back
 *     to 1000/2000);
 *   - COLORMAP_TURBO / COLORMAP_JET tables: OpenCV's colormap.cpp arrays are not in the image; the
 *     tables here follow the published definitions (Google's Turbo polynomial, the classic
 *     piecewise-linear jet), so colours may differ from OpenCV's by a few levels.  The kernels take
 *     the table as an argument; the same bytes drive both sides of the parity tests.
 */
#include "display_oracle.h"

#include <math.h>
#include <string.h>

static inline int cv_round_f(float v)
{
    if (!(v > -2147483648.f && v < 2147483648.f)) return (int)0x80000000u; /* integer indefinite */
    return (int)lrintf(v);                                                  /* half to even */
}
static inline uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

static double clamp01(double v) { return v < 0 ? 0 : v > 1 ? 1 : v; }

int orc_colormap_lut(int colormap, uint8_t lut[768])
{
    for (int i = 0; i < 256; i++) {
        const double x = i / 255.0;
        double r, g, b;
        if (colormap == ORC_COLORMAP_JET) {
            r = clamp01(1.5 - fabs(4.0 * x - 3.0));
            g = clamp01(1.5 - fabs(4.0 * x - 2.0));
            b = clamp01(1.5 - fabs(4.0 * x - 1.0));
        } else if (colormap == ORC_COLORMAP_TURBO) {
            r = 0.13572138 + x * (4.61539260 + x * (-42.66032258 + x * (132.13108234 + x * (-152.94239396 + x * 59.28637943))));
            g = 0.09140261 + x * (2.19418839 + x * (4.84296658 + x * (-14.18503333 + x * (4.27729857 + x * 2.82956604))));
            b = 0.10667330 + x * (12.64194608 + x * (-60.58204836 + x * (110.36276771 + x * (-89.90310912 + x * 27.34824973))));
            r = clamp01(r); g = clamp01(g); b = clamp01(b);
        } else {
            return -1;
        }
        lut[3 * i + 0] = (uint8_t)floor(255.0 * b + 0.5);
        lut[3 * i + 1] = (uint8_t)floor(255.0 * g + 0.5);
        lut[3 * i + 2] = (uint8_t)floor(255.0 * r + 0.5);
    }
    return 0;
}

static inline uint8_t add_weighted(uint8_t a, float alpha, uint8_t b, float beta, float gamma)
{
    return sat_u8(cv_round_f(fmaf((float)a, alpha, (float)b * beta) + gamma));
}

void orc_add_weighted_u8(const uint8_t* a, double alpha, const uint8_t* b, double beta,
                         double gamma, size_t n, uint8_t* out)
{
    for (size_t i = 0; i < n; i++) out[i] = add_weighted(a[i], (float)alpha, b[i], (float)beta, (float)gamma);
}

void orc_show_disparity_map(const float* disp, int width, int height, int num_disp,
                            const uint8_t* prev, uint8_t* out)
{
    const float scale = 1.0f / (float)(num_disp > 1 ? num_disp : 1); /* 1.0f / std::max(1, numDisp) */
    const float alpha = 0.63f;
    for (size_t i = 0; i < (size_t)width * height; i++) {
        const float d = disp[i];
        const float masked = d > 0.f ? d : 0.f;            /* setTo(0, ~(disparity > 0)) */
        const float n01 = masked * scale;                    /* convertTo(CV_32F, scale) */
        const float g = (float)pow((double)n01, 0.6);        /* cv::pow(norm01, 0.6) */
        uint8_t s = sat_u8(cv_round_f(g * 255.0f));          /* convertTo(CV_8U, 255.0) */
        if (prev) s = add_weighted(prev[i], alpha, s, 1.0f - alpha, 0.f);
        out[i] = s;
    }
}

void orc_depth_range_update(const float* xyz, int width, int height, int channels,
                            double zrange[2], float* scale, float* shift)
{
    double zmin_raw = 0, zmax_raw = 0;
    int found = 0;
    for (size_t i = 0; i < (size_t)width * height; i++) {
        const float z = xyz[i * channels + (channels == 3 ? 2 : 0)];
        if (z > 0.f && z < 10000.f && z == z) {
            if (!found || z < zmin_raw) zmin_raw = z;
            if (!found || z > zmax_raw) zmax_raw = z;
            found = 1;
        }
    }
    if (!(zmax_raw > zmin_raw)) {
        zmin_raw = 1000.0;
        zmax_raw = 2000.0;
    }
    const double a = 0.1;
    double zmin = (1.0 - a) * zrange[0] + a * zmin_raw;
    double zmax = (1.0 - a) * zrange[1] + a * zmax_raw;
    zmin = fmax(0.0, fmin(zmin, 10000.0));
    zmax = fmax(zmin + 1.0, fmin(zmax, 10000.0));
    zrange[0] = zmin;
    zrange[1] = zmax;
    *scale = (float)(255.0 / (zmax - zmin));
    *shift = (float)(-255.0 * zmin / (zmax - zmin));
}

void orc_apply_colormap(const uint8_t* src, size_t n, const uint8_t* lut, uint8_t* out)
{
    for (size_t i = 0; i < n; i++) memcpy(out + 3 * i, lut + 3 * src[i], 3);
}

void orc_show_depth_map(const float* xyz, int width, int height, int channels, double zrange[2],
                        const uint8_t* lut, const uint8_t* prev, uint8_t* out)
{
    float a, b;
    orc_depth_range_update(xyz, width, height, channels, zrange, &a, &b);
    const float alpha = 0.63f;
    for (size_t i = 0; i < (size_t)width * height; i++) {
        const float z = xyz[i * channels + (channels == 3 ? 2 : 0)];
        const uint8_t v = sat_u8(cv_round_f(fmaf(z, a, b)));  /* convertTo(CV_8U, scale, shift) */
        for (int c = 0; c < 3; c++) {
            uint8_t o = lut[3 * v + c];                         /* applyColorMap(TURBO) */
            if (prev) o = add_weighted(prev[3 * i + c], alpha, o, 1.0f - alpha, 0.f);
            out[3 * i + c] = o;
        }
    }
}

void orc_resize_area_half_bgr(const uint8_t* src, int width, int height, size_t stride, uint8_t* dst)
{
    const int dw = width / 2, dh = height / 2;
    for (int y = 0; y < dh; y++) {
        const uint8_t* a = src + (size_t)(2 * y) * stride;
        const uint8_t* b = a + stride;
        for (int x = 0; x < dw; x++)
            for (int c = 0; c < 3; c++)
                dst[((size_t)y * dw + x) * 3 + c] = (uint8_t)(
                    (a[6 * x + c] + a[6 * x + 3 + c] + b[6 * x + c] + b[6 * x + 3 + c] + 2) >> 2);
    }
}

double orc_depth_coverage(const float* xyz, int width, int height, int col0)
{
    long counter = 0;
    for (int i = 0; i < height; i++)
        for (int j = col0; j < width; j++) {
            const float z = xyz[((size_t)i * width + j) * 3 + 2];
            if (z >= 0.0 && z <= 12000.0 && !isnan(z)) counter++;
        }
    return ((double)counter / (width * height)) * 100;
}

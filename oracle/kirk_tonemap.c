/*
 * kirk_tonemap.c -- TEST INFRASTRUCTURE ONLY (see kirk_oracle.h).
 *
 * Sequential CPU restatement of KIRK's output stage, the checker for
 * khp_read_rgba8:
 *   Texture::toByte / setPixel           Common/Texture.h:252-254, Texture.cpp:222-241
 *   PathTracer::applyToneMapping         CPU/CPU_Raytracer/CPU_PathTracer.cpp:92-104
 *   Tonemapper::map and its stages       Utils/Tonemapping.cpp:9-45, 66-245
 *
 * Float/double follows the reference's expressions as its (MSVC) build
 * resolves them: float arguments take the float overloads of exp/log/pow/
 * log10, literals like 2.3e-5 and 1.099 promote to double, and the
 * log-luminance sum is a float running sum, as RGB_to_Yxy writes it.
 *
 * The per-pixel CRT calls (log, pow and their float overloads) are the
 * documented replacements ko_log_d / ko_exp_d / ko_pow_d below -- the same
 * algorithm as the product's kmath.h k_log_d / k_exp_d / k_pow_d, like every
 * other libm function on the path -- so the 8-bit output is
 * byte-identical.  The once-per-image scalars (exp/log/log10 of the two
 * reductions, the Gaussian mask) use the host libm, as the product's host
 * code does.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "kirk_oracle.h"

static const float KO_EPS = 1e-06f;      /* Tonemapping.h:12 */
static const float KO_LOG05 = -0.693147f; /* Tonemapping.h:13 */
static const float RGB2YXY[3][3] = {{0.5141364f, 0.3238786f, 0.16036376f},
                                    {0.265068f, 0.67023428f, 0.06409157f},
                                    {0.0241188f, 0.1228178f, 0.84442666f}}; /* Tonemapping.h:35-38 */
static const float YXY2RGB[3][3] = {{2.5651f, -1.1665f, -0.3986f},
                                    {-1.0217f, 1.9777f, 0.0439f},
                                    {0.0753f, -0.2543f, 1.1892f}}; /* Tonemapping.h:39-42 */

static float gdot(const float a[3], const float b[3]) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }

/* ---- double log / exp / pow: x = m 2^e with log m = 2 atanh((m-1)/(m+1)); exp by
 * x = k ln2 + r and the Taylor series of e^r to r^14; pow with C99 Annex F special
 * cases and exp(y log x).  Plain double arithmetic (-ffp-contract=off). */
static double d_bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static uint64_t bits_d(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
#define KO_LN2_HI 6.93147180369123816490e-01
#define KO_LN2_LO 1.90821492927058770002e-10
#define KO_INV_LN2 1.44269504088896338700e+00

double ko_log_d(double x) {
    if (!(x > 0.0)) return x == 0.0 ? -d_bits(0x7ff0000000000000ull) : d_bits(0x7ff8000000000000ull);
    if (x == d_bits(0x7ff0000000000000ull)) return x;
    int e = 0;
    if (x < 2.2250738585072014e-308) { x = x * 18014398509481984.0; e = -54; }
    uint64_t b = bits_d(x);
    e += (int)((b >> 52) & 0x7ffu) - 1023;
    double m = d_bits((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
    if (m > 1.41421356237309504880) { m = m * 0.5; e += 1; }
    double f = m - 1.0, s = f / (m + 1.0), z = s * s;
    static const double inv_odd[12] = {1.0 / 25.0, 1.0 / 23.0, 1.0 / 21.0, 1.0 / 19.0, 1.0 / 17.0, 1.0 / 15.0,
                                       1.0 / 13.0, 1.0 / 11.0, 1.0 / 9.0, 1.0 / 7.0, 1.0 / 5.0, 1.0 / 3.0};
    double p = inv_odd[0];
    for (int k = 1; k < 12; ++k) p = p * z + inv_odd[k];
    double lm = 2.0 * s + (2.0 * s) * (z * p);
    double de = (double)e;
    return de * KO_LN2_HI + (de * KO_LN2_LO + lm);
}

double ko_exp_d(double x) {
    if (x != x) return x;
    if (x > 709.782712893384) return d_bits(0x7ff0000000000000ull);
    if (x < -745.2) return 0.0;
    double kd = (double)(int64_t)((x * KO_INV_LN2) + (x < 0.0 ? -0.5 : 0.5));
    int k = (int)kd;
    double r = (x - kd * KO_LN2_HI) - kd * KO_LN2_LO;
    static const double inv_fact[15] = {1.0 / 87178291200.0, 1.0 / 6227020800.0, 1.0 / 479001600.0,
                                        1.0 / 39916800.0, 1.0 / 3628800.0, 1.0 / 362880.0, 1.0 / 40320.0,
                                        1.0 / 5040.0, 1.0 / 720.0, 1.0 / 120.0, 1.0 / 24.0, 1.0 / 6.0, 0.5,
                                        1.0, 1.0};
    double p = inv_fact[0];
    for (int i = 1; i < 15; ++i) p = p * r + inv_fact[i];
    if (k < -1021) return (p * d_bits((uint64_t)(k + 1023 + 54) << 52)) * (1.0 / 18014398509481984.0);
    if (k > 1023) return (p * 2.0) * d_bits((uint64_t)(k - 1 + 1023) << 52);
    return p * d_bits((uint64_t)(k + 1023) << 52);
}

static int ko_is_int(double y) { return y == (double)(int64_t)y || y > 9007199254740992.0 || y < -9007199254740992.0; }
static int ko_is_odd(double y) {
    if (y > 9007199254740992.0 || y < -9007199254740992.0) return 0;
    int64_t i = (int64_t)y;
    return (double)i == y && (i & 1);
}

double ko_pow_d(double x, double y) {
    double INF = d_bits(0x7ff0000000000000ull), NANV = d_bits(0x7ff8000000000000ull);
    if (y == 0.0) return 1.0;
    if (x == 1.0) return 1.0;
    if (x != x || y != y) return NANV;
    double ax = x < 0.0 ? -x : x;
    if (y == INF || y == -INF) {
        if (ax == 1.0) return 1.0;
        return ((ax > 1.0) == (y > 0.0)) ? INF : 0.0;
    }
    int odd = ko_is_odd(y);
    if (x == 0.0) {
        int neg = (int)(bits_d(x) >> 63);
        if (y < 0.0) return (odd && neg) ? -INF : INF;
        return (odd && neg) ? x : 0.0;
    }
    if (ax == INF) {
        if (x > 0.0) return y < 0.0 ? 0.0 : INF;
        if (y < 0.0) return odd ? -0.0 : 0.0;
        return odd ? -INF : INF;
    }
    if (x < 0.0) {
        if (!ko_is_int(y)) return NANV;
        double r = ko_exp_d(y * ko_log_d(ax));
        return odd ? -r : r;
    }
    return ko_exp_d(y * ko_log_d(x));
}
static float ko_logf_d(float x) { return (float)ko_log_d((double)x); }
static float ko_powf_d(float x, float y) { return (float)ko_pow_d((double)x, (double)y); }

/* Texture.h:252-254: std::max(std::min(f * 255.f, 255.f), 0.0f) converted to
 * unsigned char; NaN survives both and converts to 0 on x86 (cvttss2si). */
static uint8_t to_byte(float f) {
    float a = f * 255.0f;
    float lo = (255.0f < a) ? 255.0f : a;
    float v = (lo < 0.0f) ? 0.0f : lo;
    return (v == v) ? (uint8_t)(uint32_t)v : 0;
}

void ko_tonemap_defaults(khp_tonemap* t) {
    memset(t, 0, sizeof(*t));
    t->bias = 0.85f;
    t->gamma = 1.0f;
    t->white = 1.0f;
    t->kernel_multiplier = 0.125f;
    t->center_x = t->center_y = -1;
}

/* rgb (W*H*3) -> rgba (W*H*4), Texture::setPixel(vec4(rgb, 1)) per pixel. */
void ko_to_rgba8(uint32_t n, const float* rgb, uint8_t* out) {
    for (uint32_t i = 0; i < n; ++i) {
        out[4 * i] = to_byte(rgb[3 * i]);
        out[4 * i + 1] = to_byte(rgb[3 * i + 1]);
        out[4 * i + 2] = to_byte(rgb[3 * i + 2]);
        out[4 * i + 3] = to_byte(1.0f);
    }
}

/* Tonemapper::luminance_from_center (Tonemapping.cpp:183-245), literally,
 * including its i1 = x * (y_start + kernel_size) + y indexing.  Returns -1
 * when that index would leave the image (the reference reads out of bounds). */
static int center_world_lum(const float* img, int width, int height, float km, int cx, int cy, float* world_lum) {
    int ks = width < height ? (int)(width * km) : (int)(height * km);
    if (ks > width || ks > height) ks = width < height ? width : height;
    else if (ks < 1) ks = 1;
    if (ks % 2 == 0) ks -= 1;
    int half = (int)floor(ks * 0.5);
    int xs, ys;
    if (cx + half > width) xs = width - ks;
    else if (cx - half < 0) xs = 0;
    else xs = cx - half;
    if (cy + half > height) ys = height - ks;
    else if (cy - half < 0) ys = 0;
    else ys = cy - half;
    if ((long)(xs + ks) * (ys + ks) > (long)width * height || xs < 0 || ys < 0) return -1;
    double* mask = (double*)malloc(sizeof(double) * (size_t)ks * ks);
    double acc = 0.0;
    for (int idx = 0; idx < ks * ks; ++idx) {
        int x = idx % ks - half, y = idx / ks - half;
        float r = (float)sqrt((double)(x * x + y * y));
        mask[idx] = exp(-log(2.0) * pow((double)(r / (float)half), 2.0));
    }
    for (int idx = 0; idx < ks * ks; ++idx) acc += mask[idx];
    double mean = (double)(ks * ks) / acc;
    double sum = 0.0;
    for (int x = xs, i = 0; x < xs + ks; x++, i++)
        for (int y = ys, j = 0; y < ys + ks; y++, j++) {
            int i1 = x * (ys + ks) + y;
            int i2 = j * ks + i;
            sum += ko_log_d(2.3e-5 + (double)img[3 * (size_t)i1] * mask[i2] * mean);
        }
    free(mask);
    *world_lum = (float)(sum / (ks * ks));
    return 0;
}

/* Tonemapper::map on rgb (W*H*3, in place semantics: out_rgb may alias rgb).
 * max_lum / world_lum: the two reductions (may be NULL).  Returns 0, or -1
 * for a center window outside the image. */
int ko_tonemap(uint32_t W, uint32_t H, const float* rgb, const khp_tonemap* tm, float* out_rgb, float* max_lum_out,
               float* world_lum_out) {
    const size_t n = (size_t)W * H;
    float* img = (float*)malloc(sizeof(float) * 3 * (n ? n : 1));
    memcpy(img, rgb, sizeof(float) * 3 * n);
    /* map: Tonemapping.cpp:11-18, 21 */
    int cx = tm->center_x < 0 ? (int)W / 2 : tm->center_x;
    int cy = tm->center_y < 0 ? (int)H / 2 : tm->center_y;
    float exposure = (float)pow(2.0, (double)tm->exposure);
    /* RGB_to_Yxy: Tonemapping.cpp:66-91 */
    float mx = KO_EPS, sum = 0.0f;
    for (size_t i = 0; i < n; ++i) {
        float* v = img + 3 * i;
        float res[3] = {gdot(RGB2YXY[0], v), gdot(RGB2YXY[1], v), gdot(RGB2YXY[2], v)};
        float one[3] = {1.0f, 1.0f, 1.0f};
        float Wt = gdot(res, one);
        if (Wt > 0.0f) {
            v[0] = res[1];
            v[1] = res[0] / Wt;
            v[2] = res[1] / Wt;
        } else {
            v[0] = v[1] = v[2] = 0.0f;
        }
        mx = (mx < v[0]) ? v[0] : mx;
        sum = (float)((double)sum + ko_log_d(2.3e-5 + (double)v[0]));
    }
    float world_lum = sum / (float)n;
    if (tm->center_weight) {
        if (center_world_lum(img, (int)W, (int)H, tm->kernel_multiplier, cx, cy, &world_lum)) {
            free(img);
            return -1;
        }
    }
    if (max_lum_out) *max_lum_out = mx;
    if (world_lum_out) *world_lum_out = world_lum;
    /* tonemapping: Tonemapping.cpp:116-144 */
    float av_lum = expf(world_lum) / 1.0f;
    float biasP = logf(tm->bias) / KO_LOG05;
    float contP = 1.0f / tm->contrast;
    float Lmax = mx / av_lum;
    float divider = log10f(Lmax + 1.0f);
    for (size_t i = 0; i < n; ++i) {
        float* v = img + 3 * i;
        if (tm->contrast != 0.0f) v[0] = ko_powf_d(v[0], contP);
        v[0] /= av_lum;
        v[0] *= exposure;
        float b = (float)ko_pow_d((double)(v[0] / Lmax), (double)biasP); /* Tonemapper::bias, Tonemapping.h:51-54 */
        float interpol = ko_logf_d(2.0f + b * 8.0f);
        v[0] = ko_logf_d(v[0] + 1.0f) / interpol / divider;
    }
    /* Yxy_to_RGB: Tonemapping.cpp:93-114 */
    for (size_t i = 0; i < n; ++i) {
        float* v = img + 3 * i;
        float Y = v[0], x = v[1], y = v[2], X, Z;
        if (Y > KO_EPS && x > KO_EPS && y > KO_EPS) {
            X = x * Y / y;
            Z = X / x - X - Y;
        } else {
            X = Z = KO_EPS;
        }
        float xyz[3] = {X, Y, Z};
        v[0] = gdot(YXY2RGB[0], xyz);
        v[1] = gdot(YXY2RGB[1], xyz);
        v[2] = gdot(YXY2RGB[2], xyz);
    }
    /* gamma: Tonemapping.cpp:31-37, 146-181 */
    if ((double)tm->gamma != 1.0) {
        if (tm->rec_gamma) {
            float inv_gamma = (float)(0.45 / (double)tm->gamma * 2.0);
            float slope = 4.5f, start = 0.018f;
            if ((double)tm->gamma >= 2.1) {
                start = (float)(0.018 / ((double)(tm->gamma - 2.0f) * 7.5));
                slope = (float)(4.5 * ((double)(tm->gamma - 2.0f) * 7.5));
            } else if ((double)tm->gamma <= 1.9) {
                start = (float)(0.018 * ((double)(2.0f - tm->gamma) * 7.5));
                slope = (float)(4.5 / ((double)(2.0f - tm->gamma) * 7.5));
            }
            for (size_t k = 0; k < 3 * n; ++k)
                img[k] = img[k] <= start ? img[k] * slope : (float)(1.099 * (double)ko_powf_d(img[k], inv_gamma) - 0.099);
        } else {
            float inv_gamma = 1.0f / tm->gamma;
            for (size_t k = 0; k < 3 * n; ++k) img[k] = ko_powf_d(img[k], inv_gamma);
        }
    }
    /* clamp: Tonemapping.cpp:38-44 (glm::clamp = min(max(x, lo), hi)) */
    if (tm->white != 1.0f || tm->black != 0.0f)
        for (size_t k = 0; k < 3 * n; ++k) {
            float c = (img[k] < tm->black) ? tm->black : img[k];
            img[k] = (tm->white < c) ? tm->white : c;
        }
    memcpy(out_rgb, img, sizeof(float) * 3 * n);
    free(img);
    return 0;
}

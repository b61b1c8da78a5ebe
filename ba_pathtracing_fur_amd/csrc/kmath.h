// kmath.h -- numeric definitions shared by the host flatten/BVH code and the
// gfx950 kernels.  Every function is plain IEEE float arithmetic (build with
// -ffp-contract=off, correctly-rounded sqrt/div, denormals kept), so host and
// device produce identical bits.  The definitions are the ones DESIGN.md
// documents under "kmath" (Cephes-style polynomials, J0 power series); KIRK
// itself used GLM + the platform libm.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define KHD __host__ __device__ __forceinline__
#else
#include <math.h>
#define KHD static inline
#endif

namespace khp {

constexpr float PIF = 3.14159265358979323846f;
constexpr float PIO2F = 1.57079632679489661923f;
constexpr float PIO4F = 0.785398163397448309616f;
constexpr float ONE_OVER_PI = 0.318309886183790671537767526745028724f;  // glm::one_over_pi<float>
constexpr float HALF_PI = 1.57079632679489661923132169163975144f;       // glm::half_pi<float>
constexpr float QUARTER_PI = 0.785398163397448309615660845819875721f;   // glm::quarter_pi<float>
constexpr double M_PI_D = 3.14159265358979323846;                        // M_PI
constexpr float DEG2RAD = 0.01745329251994329576923690768489f;          // glm::radians
constexpr float RAD2DEG = 57.295779513082320876798154814105f;           // glm::degrees
constexpr float FLT_MAX_ = 3.402823466e+38F;
constexpr float FLT_EPS_ = 1.192092896e-07F;

KHD float f_from_bits(uint32_t u) {
    union { uint32_t u; float f; } c;
    c.u = u;
    return c.f;
}
KHD uint32_t bits_from_f(float f) {
    union { float f; uint32_t u; } c;
    c.f = f;
    return c.u;
}
KHD float k_sqrt(float x) { return sqrtf(x); }
KHD float k_fabs(float x) { return fabsf(x); }
KHD bool k_isnan(float x) { return x != x; }
KHD float k_nan() { return f_from_bits(0x7fc00000u); }
KHD float k_inf() { return f_from_bits(0x7f800000u); }

KHD float k_ldexpf(float x, int n) {
    if (n > 127) {
        x = x * f_from_bits((uint32_t)(127 + 127) << 23);
        n -= 127;
        if (n > 127) n = 127;
    } else if (n < -126) {
        x = x * f_from_bits((uint32_t)1 << 23);
        n += 126;
        if (n < -126) n = -126;
    }
    return x * f_from_bits((uint32_t)(n + 127) << 23);
}

KHD float k_sin_poly(float z, float x) {
    float y = ((-1.9515295891E-4f * z + 8.3321608736E-3f) * z - 1.6666654611E-1f) * z * x;
    return y + x;
}
KHD float k_cos_poly(float z) {
    float y = ((2.443315711809948E-005f * z - 1.388731625493765E-003f) * z + 4.166664568298827E-002f) * z * z;
    y = y - 0.5f * z;
    return y + 1.0f;
}
constexpr float DP1 = 0.78515625f;
constexpr float DP2 = 2.4187564849853515625e-4f;
constexpr float DP3 = 3.77489497744594108e-8f;
constexpr float FOPI = 1.27323954473516f;

KHD float k_sinf(float x) {
    if (k_isnan(x)) return x;
    bool neg = false;
    if (x < 0.0f) { neg = true; x = -x; }
    int j = (int)(FOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { neg = !neg; j -= 4; }
    x = ((x - y * DP1) - y * DP2) - y * DP3;
    float z = x * x;
    y = (j == 1 || j == 2) ? k_cos_poly(z) : k_sin_poly(z, x);
    return neg ? -y : y;
}

KHD float k_cosf(float x) {
    if (k_isnan(x)) return x;
    bool neg = false;
    if (x < 0.0f) x = -x;
    int j = (int)(FOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { j -= 4; neg = !neg; }
    if (j > 1) neg = !neg;
    x = ((x - y * DP1) - y * DP2) - y * DP3;
    float z = x * x;
    y = (j == 1 || j == 2) ? k_sin_poly(z, x) : k_cos_poly(z);
    return neg ? -y : y;
}

KHD float k_atanf(float x) {
    bool neg = false;
    float y;
    if (x < 0.0f) { neg = true; x = -x; }
    if (x > 2.414213562373095f) { y = PIO2F; x = -(1.0f / x); }
    else if (x > 0.4142135623730950f) { y = PIO4F; x = (x - 1.0f) / (x + 1.0f); }
    else y = 0.0f;
    float z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032E-1f) * z + 1.99777106478E-1f) * z - 3.33329491539E-1f) * z * x + x);
    return neg ? -y : y;
}

KHD float k_atan2f(float y, float x) {
    if (k_isnan(x) || k_isnan(y)) return x + y;
    int code = 0;
    if (x < 0.0f) code = 2;
    if (y < 0.0f) code |= 1;
    if (x == 0.0f) {
        if (code & 1) return -PIO2F;
        if (y == 0.0f) return 0.0f;
        return PIO2F;
    }
    if (y == 0.0f) return (code & 2) ? PIF : 0.0f;
    float w = 0.0f;
    if (code == 2) w = PIF;
    else if (code == 3) w = -PIF;
    return w + k_atanf(y / x);
}

KHD float k_asinf(float x) {
    if (k_isnan(x)) return x;
    bool neg = false;
    float a = x, z;
    if (x < 0.0f) { neg = true; a = -x; }
    if (a > 1.0f) return k_nan();
    if (a < 1.0e-4f) {
        z = a;
    } else {
        float xx;
        bool flag = false;
        if (a > 0.5f) { z = 0.5f * (1.0f - a); xx = sqrtf(z); flag = true; }
        else { xx = a; z = xx * xx; }
        z = ((((4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z + 7.4953002686E-2f) * z
             + 1.6666752422E-1f) * z * xx + xx;
        if (flag) { z = z + z; z = PIO2F - z; }
    }
    return neg ? -z : z;
}

KHD float k_acosf(float x) {
    if (k_isnan(x)) return x;
    if (x < -1.0f || x > 1.0f) return k_nan();
    if (x < -0.5f) return PIF - 2.0f * k_asinf(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * k_asinf(sqrtf(0.5f * (1.0f - x)));
    return PIO2F - k_asinf(x);
}

KHD float k_expf(float x) {
    if (k_isnan(x)) return x;
    if (x > 88.72283905206835f) return k_inf();
    if (x < -103.278929903431851103f) return 0.0f;
    float z = floorf(1.44269504088896341f * x + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    int n = (int)z;
    z = x * x;
    z = (((((1.9875691500E-4f * x + 1.3981999507E-3f) * x + 8.3334519073E-3f) * x + 4.1665795894E-2f) * x
          + 1.6666665459E-1f) * x + 5.0000001201E-1f) * z + x + 1.0f;
    return k_ldexpf(z, n);
}

KHD float k_sinhf(float x) {
    float a = x < 0.0f ? -x : x;
    float z;
    if (a > 1.0f) {
        z = k_expf(a);
        z = 0.5f * z - (0.5f / z);
        return x < 0.0f ? -z : z;
    }
    z = x * x;
    return ((2.03721912945E-4f * z + 8.33028376239E-3f) * z + 1.66667160211E-1f) * z * x + x;
}

// Bessel J0 by its power series, 40 terms, double (replaces MSVC _j0).
KHD double k_j0(double x) {
    double q = -0.25 * x * x, term = 1.0, sum = 1.0;
    for (int k = 1; k <= 40; ++k) {
        term = term * q / ((double)k * (double)k);
        sum = sum + term;
    }
    return sum;
}

KHD float k_hypotf(float x, float y) { return sqrtf(x * x + y * y); }

// ---- double log / exp / pow (the output stage's libm calls: Tonemapping.cpp) ----
// Plain IEEE double arithmetic (no FMA contraction), identical on host, device
// and in oracle/ (ko_log_d / ko_exp_d / ko_pow_d), within ~1 ulp of the
// correctly rounded value (tests/test_kmath.py).
KHD double d_from_bits(uint64_t u) {
    union { uint64_t u; double d; } c;
    c.u = u;
    return c.d;
}
KHD uint64_t bits_from_d(double d) {
    union { double d; uint64_t u; } c;
    c.d = d;
    return c.u;
}
constexpr double LN2_HI_D = 6.93147180369123816490e-01;  // ln 2, high part (trailing zeros: k*LN2_HI exact)
constexpr double LN2_LO_D = 1.90821492927058770002e-10;
constexpr double INV_LN2_D = 1.44269504088896338700e+00;

// log x: x = m 2^e, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m-1)/(m+1).
KHD double k_log_d(double x) {
    if (!(x > 0.0)) return x == 0.0 ? -d_from_bits(0x7ff0000000000000ull) : d_from_bits(0x7ff8000000000000ull);
    if (x == d_from_bits(0x7ff0000000000000ull)) return x;
    int e = 0;
    if (x < 2.2250738585072014e-308) {  // subnormal
        x = x * 18014398509481984.0;    // 2^54
        e = -54;
    }
    uint64_t b = bits_from_d(x);
    e += (int)((b >> 52) & 0x7ffu) - 1023;
    double m = d_from_bits((b & 0x000fffffffffffffull) | 0x3ff0000000000000ull);
    if (m > 1.41421356237309504880) {
        m = m * 0.5;
        e += 1;
    }
    const double f = m - 1.0, s = f / (m + 1.0), z = s * s;
    double p = 1.0 / 25.0;
    p = p * z + 1.0 / 23.0;
    p = p * z + 1.0 / 21.0;
    p = p * z + 1.0 / 19.0;
    p = p * z + 1.0 / 17.0;
    p = p * z + 1.0 / 15.0;
    p = p * z + 1.0 / 13.0;
    p = p * z + 1.0 / 11.0;
    p = p * z + 1.0 / 9.0;
    p = p * z + 1.0 / 7.0;
    p = p * z + 1.0 / 5.0;
    p = p * z + 1.0 / 3.0;
    const double lm = 2.0 * s + (2.0 * s) * (z * p);
    const double de = (double)e;
    return de * LN2_HI_D + (de * LN2_LO_D + lm);
}

// exp x: x = k ln2 + r, |r| <= ln2/2, Taylor series of e^r to r^14, times 2^k.
KHD double k_exp_d(double x) {
    if (x != x) return x;
    if (x > 709.782712893384) return d_from_bits(0x7ff0000000000000ull);
    if (x < -745.2) return 0.0;
    const double kd = (double)(int64_t)((x * INV_LN2_D) + (x < 0.0 ? -0.5 : 0.5));
    const int k = (int)kd;
    const double r = (x - kd * LN2_HI_D) - kd * LN2_LO_D;
    double p = 1.0 / 87178291200.0;          // 1/14!
    p = p * r + 1.0 / 6227020800.0;          // 1/13!
    p = p * r + 1.0 / 479001600.0;
    p = p * r + 1.0 / 39916800.0;
    p = p * r + 1.0 / 3628800.0;
    p = p * r + 1.0 / 362880.0;
    p = p * r + 1.0 / 40320.0;
    p = p * r + 1.0 / 5040.0;
    p = p * r + 1.0 / 720.0;
    p = p * r + 1.0 / 120.0;
    p = p * r + 1.0 / 24.0;
    p = p * r + 1.0 / 6.0;
    p = p * r + 0.5;
    p = p * r + 1.0;
    p = p * r + 1.0;
    if (k < -1021) return (p * d_from_bits((uint64_t)(k + 1023 + 54) << 52)) * (1.0 / 18014398509481984.0);
    if (k > 1023) return (p * 2.0) * d_from_bits((uint64_t)(k - 1 + 1023) << 52);
    return p * d_from_bits((uint64_t)(k + 1023) << 52);
}

// pow with C99 Annex F special cases; finite positive x: exp(y log x).
KHD bool k_is_int_d(double y) { return y == (double)(int64_t)y || (y > 9007199254740992.0 || y < -9007199254740992.0); }
KHD bool k_is_odd_d(double y) {
    if (y > 9007199254740992.0 || y < -9007199254740992.0) return false;
    const int64_t i = (int64_t)y;
    return (double)i == y && (i & 1);
}
KHD double k_pow_d(double x, double y) {
    const double INF = d_from_bits(0x7ff0000000000000ull), NAN_ = d_from_bits(0x7ff8000000000000ull);
    if (y == 0.0) return 1.0;
    if (x == 1.0) return 1.0;
    if (x != x || y != y) return NAN_;
    const double ax = x < 0.0 ? -x : x;
    if (y == INF || y == -INF) {
        if (ax == 1.0) return 1.0;
        return ((ax > 1.0) == (y > 0.0)) ? INF : 0.0;
    }
    const bool odd = k_is_odd_d(y);
    if (x == 0.0) {
        const bool neg = bits_from_d(x) >> 63;
        if (y < 0.0) return (odd && neg) ? -INF : INF;
        return (odd && neg) ? x : 0.0;
    }
    if (ax == INF) {
        if (x > 0.0) return y < 0.0 ? 0.0 : INF;
        if (y < 0.0) return odd ? -0.0 : 0.0;
        return odd ? -INF : INF;
    }
    if (x < 0.0) {
        if (!k_is_int_d(y)) return NAN_;
        const double r = k_exp_d(y * k_log_d(ax));
        return odd ? -r : r;
    }
    return k_exp_d(y * k_log_d(x));
}
// float overloads as the C++ <cmath> calls std::log(float) / std::pow(float, float)
KHD float k_logf_d(float x) { return (float)k_log_d((double)x); }
KHD float k_powf_d(float x, float y) { return (float)k_pow_d((double)x, (double)y); }

// ---- counter RNG (DESIGN.md "RNG") ----------------------------------------
KHD uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
KHD uint32_t path_key(uint32_t seed, uint32_t pixel, uint32_t sample) {
    return lowbias32(lowbias32(lowbias32(seed ^ 0x4B49524Bu) ^ pixel) + sample * 0x9E3779B9u);
}
KHD uint32_t draw_u32(uint32_t key, uint32_t dim) { return lowbias32(key ^ (dim * 0x85EBCA6Bu + 0x632BE5ABu)); }
KHD float draw_u01(uint32_t key, uint32_t dim) { return (float)(draw_u32(key, dim) >> 8) * (1.0f / 16777216.0f); }

enum Purpose : uint32_t {
    P_CAM_X = 0, P_CAM_Y = 1, P_BSDF_0 = 2, P_BSDF_1 = 3, P_LIGHT_SEL = 4, P_LIGHT_0 = 5, P_LIGHT_1 = 6,
    P_HAIR_ALPHA = 7, P_HAIR_BETA = 8
};
KHD uint32_t dim_of(uint32_t bounce, uint32_t purpose) { return bounce * 16u + purpose; }

// ---- GLM-equivalent vector algebra (GLM 0.9.9 operand order) ---------------
struct v3 {
    float x, y, z;
};
KHD v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
KHD v3 operator+(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
KHD v3 operator-(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
KHD v3 operator-(v3 a) { return mk(-a.x, -a.y, -a.z); }
KHD v3 operator*(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
KHD v3 operator*(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
KHD v3 operator/(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
KHD float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
KHD v3 cross(v3 a, v3 b) { return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
KHD float length(v3 a) { return sqrtf(dot(a, a)); }
KHD v3 normalize(v3 a) { return a * (1.0f / sqrtf(dot(a, a))); }
KHD float gmin(float x, float y) { return (y < x) ? y : x; }
KHD float gmax(float x, float y) { return (x < y) ? y : x; }
KHD float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
KHD v3 vmin(v3 a, v3 b) { return mk(gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)); }
KHD v3 vmax(v3 a, v3 b) { return mk(gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)); }
KHD bool is_zero(v3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
KHD float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
KHD v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
KHD v3 faceforward(v3 N, v3 I, v3 Nref) { return dot(Nref, I) < 0.0f ? N : -N; }
KHD v3 reflect(v3 I, v3 N) { return I - (N * dot(N, I)) * 2.0f; }
KHD v3 refract(v3 I, v3 N, float eta) {
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (!(k >= 0.0f)) return mk(0.0f, 0.0f, 0.0f);
    return I * eta - N * (eta * d + sqrtf(k));
}
// vec3(vec4(d,0) * glm::rotate(angle, axis)) = R^T d
KHD v3 rotate_rowvec(v3 d, float angle, v3 axis_in) {
    float c = k_cosf(angle), s = k_sinf(angle);
    v3 a = normalize(axis_in);
    v3 t = a * (1.0f - c);
    float R00 = c + t.x * a.x, R01 = t.x * a.y + s * a.z, R02 = t.x * a.z - s * a.y;
    float R10 = t.y * a.x - s * a.z, R11 = c + t.y * a.y, R12 = t.y * a.z + s * a.x;
    float R20 = t.z * a.x + s * a.y, R21 = t.z * a.y - s * a.x, R22 = c + t.z * a.z;
    return mk((R00 * d.x + R01 * d.y) + R02 * d.z, (R10 * d.x + R11 * d.y) + R12 * d.z,
              (R20 * d.x + R21 * d.y) + R22 * d.z);
}
KHD float angle(v3 x, v3 y) { return k_acosf(gclamp(dot(x, y), -1.0f, 1.0f)); }
KHD v3 world_to_local(v3 v, v3 X, v3 Y, v3 Z) { return mk(dot(v, X), dot(v, Y), dot(v, Z)); }
KHD v3 local_to_world(v3 v, v3 X, v3 Y, v3 Z) { return (X * v.x + Y * v.y) + Z * v.z; }
KHD v3 local_to_world_normal(v3 v, v3 n) {
    v3 dx0 = mk(0.0f, n.z, -n.y), dx1 = mk(-n.z, 0.0f, n.x);
    v3 s = normalize(n.y * n.y > n.x * n.x ? dx0 : dx1);
    v3 t = normalize(cross(n, s));
    return local_to_world(v, s, t, n);
}

}  // namespace khp

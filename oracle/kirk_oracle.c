/*
 * kirk_oracle.c -- TEST INFRASTRUCTURE ONLY (see kirk_oracle.h).
 *
 * Plain-C restatement of KIRK's CPU path tracer for fur scenes.  Every
 * function cites the reference lines it follows (paths relative to
 * /root/reference/src/libraries/KIRK/).  Third-party arithmetic the reference
 * pulls from outside its tree is restated from its published definition:
 *   - GLM (version unpinned, FindGLM.cmake only): dot/cross/normalize/length/
 *     reflect/refract/faceforward/rotate/angle/min/max/clamp, written with
 *     GLM 0.9.9's operand order;
 *   - libm / MSVC CRT (sin, cos, atan2, acos, asin, exp, sinh, hypot, _j0):
 *     replaced by the "kmath" definitions below (Cephes-style polynomials;
 *     Bessel J0 by its power series in double).  The product uses the same
 *     definitions, so CPU and GPU agree bit-for-bit;
 *   - std::mt19937 / std::random_device: replaced by the counter RNG below.
 * Build with -ffp-contract=off (no FMA contraction) -- see oracle/Makefile.
 */
#include "kirk_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

/* ======================================================================= */
/*  kmath: the shared numeric definitions                                   */
/* ======================================================================= */

#define K_PIF 3.14159265358979323846f
#define K_PIO2F 1.57079632679489661923f
#define K_PIO4F 0.785398163397448309616f
#define K_ONE_OVER_PI 0.318309886183790671537767526745028724f /* glm::one_over_pi<float> */
#define K_HALF_PI 1.57079632679489661923132169163975144f       /* glm::half_pi<float> */
#define K_QUARTER_PI 0.785398163397448309615660845819875721f   /* glm::quarter_pi<float> */
#define K_M_PI 3.14159265358979323846                           /* M_PI (double) */
#define K_DEG2RAD 0.01745329251994329576923690768489f           /* glm::radians */
#define K_RAD2DEG 57.295779513082320876798154814105f            /* glm::degrees */

static float k_ldexpf(float x, int n) {
    union { float f; uint32_t u; } s;
    if (n > 127) {
        s.u = (uint32_t)(127 + 127) << 23; x = x * s.f; n -= 127;
        if (n > 127) n = 127;
    } else if (n < -126) {
        s.u = (uint32_t)1 << 23; x = x * s.f; n += 126;    /* 2^-126 */
        if (n < -126) n = -126;
    }
    s.u = (uint32_t)(n + 127) << 23;
    return x * s.f;
}

/* Cephes sinf/cosf core (range reduction by 3-part pi/4). */
static float k_sin_poly(float z, float x) {
    float y = ((-1.9515295891E-4f * z + 8.3321608736E-3f) * z - 1.6666654611E-1f) * z * x;
    return y + x;
}
static float k_cos_poly(float z) {
    float y = ((2.443315711809948E-005f * z - 1.388731625493765E-003f) * z + 4.166664568298827E-002f) * z * z;
    y = y - 0.5f * z;
    return y + 1.0f;
}
#define K_DP1 0.78515625f
#define K_DP2 2.4187564849853515625e-4f
#define K_DP3 3.77489497744594108e-8f
#define K_FOPI 1.27323954473516f

float ko_sinf(float x) {
    float sign = 1.0f;
    if (x != x) return x;
    if (x < 0.0f) { sign = -1.0f; x = -x; }
    int j = (int)(K_FOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { sign = -sign; j -= 4; }
    x = ((x - y * K_DP1) - y * K_DP2) - y * K_DP3;
    float z = x * x;
    y = (j == 1 || j == 2) ? k_cos_poly(z) : k_sin_poly(z, x);
    return sign < 0.0f ? -y : y;
}

float ko_cosf(float x) {
    float sign = 1.0f;
    if (x != x) return x;
    if (x < 0.0f) x = -x;
    int j = (int)(K_FOPI * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { j -= 4; sign = -sign; }
    if (j > 1) sign = -sign;
    x = ((x - y * K_DP1) - y * K_DP2) - y * K_DP3;
    float z = x * x;
    y = (j == 1 || j == 2) ? k_sin_poly(z, x) : k_cos_poly(z);
    return sign < 0.0f ? -y : y;
}

static float k_atanf(float x) {
    float sign = 1.0f, y;
    if (x < 0.0f) { sign = -1.0f; x = -x; }
    if (x > 2.414213562373095f) { y = K_PIO2F; x = -(1.0f / x); }
    else if (x > 0.4142135623730950f) { y = K_PIO4F; x = (x - 1.0f) / (x + 1.0f); }
    else y = 0.0f;
    float z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032E-1f) * z + 1.99777106478E-1f) * z - 3.33329491539E-1f) * z * x + x);
    return sign < 0.0f ? -y : y;
}

float ko_atan2f(float y, float x) {
    if (x != x || y != y) return x + y;
    int code = 0;
    if (x < 0.0f) code = 2;
    if (y < 0.0f) code |= 1;
    if (x == 0.0f) {
        if (code & 1) return -K_PIO2F;
        if (y == 0.0f) return 0.0f;
        return K_PIO2F;
    }
    if (y == 0.0f) {
        if (code & 2) return K_PIF;
        return 0.0f;
    }
    float w = 0.0f;
    if (code == 2) w = K_PIF;
    else if (code == 3) w = -K_PIF;
    return w + k_atanf(y / x);
}

float ko_asinf(float x) {
    float sign = 1.0f, a = x, z;
    int flag = 0;
    if (x != x) return x;
    if (x < 0.0f) { sign = -1.0f; a = -x; }
    if (a > 1.0f) return NAN;
    if (a < 1.0e-4f) { z = a; }
    else {
        float xx;
        if (a > 0.5f) { z = 0.5f * (1.0f - a); xx = sqrtf(z); flag = 1; }
        else { xx = a; z = xx * xx; }
        z = ((((4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z + 7.4953002686E-2f) * z
             + 1.6666752422E-1f) * z * xx + xx;
        if (flag) { z = z + z; z = K_PIO2F - z; }
    }
    return sign < 0.0f ? -z : z;
}

float ko_acosf(float x) {
    if (x != x) return x;
    if (x < -1.0f || x > 1.0f) return NAN;
    if (x < -0.5f) return K_PIF - 2.0f * ko_asinf(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * ko_asinf(sqrtf(0.5f * (1.0f - x)));
    return K_PIO2F - ko_asinf(x);
}

float ko_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283905206835f) return INFINITY;
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

float ko_sinhf(float x) {
    float a = x < 0.0f ? -x : x;
    float z;
    if (a > 1.0f) {
        z = ko_expf(a);
        z = 0.5f * z - (0.5f / z);
        return x < 0.0f ? -z : z;
    }
    z = x * x;
    return ((2.03721912945E-4f * z + 8.33028376239E-3f) * z + 1.66667160211E-1f) * z * x + x;
}

/* Bessel J0 (MSVC _j0 at Bsdf.cpp:837,919,995): power series, 40 terms, double. */
double ko_j0(double x) {
    double q = -0.25 * x * x, term = 1.0, sum = 1.0;
    for (int k = 1; k <= 40; ++k) {
        term = term * q / ((double)k * (double)k);
        sum = sum + term;
    }
    return sum;
}

/* std::hypot(float,float) at Bsdf.cpp:511,690 -- defined as sqrt(x*x+y*y). */
static float k_hypotf(float x, float y) { return sqrtf(x * x + y * y); }

/* ======================================================================= */
/*  counter RNG (replaces every std::mt19937 draw; DESIGN.md "RNG")          */
/* ======================================================================= */
static uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
static uint32_t path_key(uint32_t seed, uint32_t pixel, uint32_t sample) {
    return lowbias32(lowbias32(lowbias32(seed ^ 0x4B49524Bu) ^ pixel) + sample * 0x9E3779B9u);
}
static uint32_t draw_u32(uint32_t key, uint32_t dim) { return lowbias32(key ^ (dim * 0x85EBCA6Bu + 0x632BE5ABu)); }
static float draw_u01(uint32_t key, uint32_t dim) { return (float)(draw_u32(key, dim) >> 8) * (1.0f / 16777216.0f); }
uint32_t ko_rand_u32(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t dim) {
    return draw_u32(path_key(seed, pixel, sample), dim);
}
/* draw purposes, dim = bounce*16 + purpose */
enum { P_CAM_X = 0, P_CAM_Y = 1, P_BSDF_0 = 2, P_BSDF_1 = 3, P_LIGHT_SEL = 4, P_LIGHT_0 = 5, P_LIGHT_1 = 6,
       P_HAIR_ALPHA = 7, P_HAIR_BETA = 8 };
#define DIM(b, p) ((uint32_t)(b) * 16u + (uint32_t)(p))

/* ======================================================================= */
/*  GLM-equivalent vector algebra (operand order of GLM 0.9.9)              */
/* ======================================================================= */
typedef struct { float x, y, z; } v3;
static v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }
static v3 vmul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static v3 vscale(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static v3 vdivs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static float dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static v3 cross(v3 a, v3 b) {
    return V(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static float length(v3 a) { return sqrtf(dot(a, a)); }
static v3 normalize(v3 a) { return vscale(a, 1.0f / sqrtf(dot(a, a))); }
static float gmin(float x, float y) { return (y < x) ? y : x; }
static float gmax(float x, float y) { return (x < y) ? y : x; }
static float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
static v3 v3min(v3 a, v3 b) { return V(gmin(a.x, b.x), gmin(a.y, b.y), gmin(a.z, b.z)); }
static v3 v3max(v3 a, v3 b) { return V(gmax(a.x, b.x), gmax(a.y, b.y), gmax(a.z, b.z)); }
static int is_zero(v3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
static float comp(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static void set_comp(v3* a, int i, float v) { if (i == 0) a->x = v; else if (i == 1) a->y = v; else a->z = v; }
static v3 ld3(const float* p) { return V(p[0], p[1], p[2]); }
/* glm::faceforward(N, I, Nref) */
static v3 faceforward(v3 N, v3 I, v3 Nref) { return dot(Nref, I) < 0.0f ? N : vneg(N); }
/* glm::reflect(I, N) = I - N * dot(N, I) * 2 */
static v3 reflect(v3 I, v3 N) { return vsub(I, vscale(vscale(N, dot(N, I)), 2.0f)); }
/* glm::refract(I, N, eta) */
static v3 refract(v3 I, v3 N, float eta) {
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (!(k >= 0.0f)) return V(0.0f, 0.0f, 0.0f);
    return vsub(vscale(I, eta), vscale(N, eta * d + sqrtf(k)));
}
/* vec3(vec4(d,0) * glm::rotate(angle, axis)) -- i.e. R^T d (Rodrigues) */
static v3 rotate_rowvec(v3 d, float angle, v3 axis_in) {
    float c = ko_cosf(angle), s = ko_sinf(angle);
    v3 a = normalize(axis_in);
    v3 t = vscale(a, 1.0f - c);
    float R00 = c + t.x * a.x, R01 = t.x * a.y + s * a.z, R02 = t.x * a.z - s * a.y;
    float R10 = t.y * a.x - s * a.z, R11 = c + t.y * a.y, R12 = t.y * a.z + s * a.x;
    float R20 = t.z * a.x + s * a.y, R21 = t.z * a.y - s * a.x, R22 = c + t.z * a.z;
    return V((R00 * d.x + R01 * d.y) + R02 * d.z, (R10 * d.x + R11 * d.y) + R12 * d.z,
             (R20 * d.x + R21 * d.y) + R22 * d.z);
}
/* glm::angle(x, y) = acos(clamp(dot(x,y), -1, 1)) */
static float angle(v3 x, v3 y) { return ko_acosf(gclamp(dot(x, y), -1.0f, 1.0f)); }
/* Math::worldToLocal / localToWorld / localToWorldNormal (Utils/Math.cpp:7-24) */
static v3 world_to_local(v3 v, v3 X, v3 Y, v3 Z) { return V(dot(v, X), dot(v, Y), dot(v, Z)); }
static v3 local_to_world(v3 v, v3 X, v3 Y, v3 Z) { return vadd(vadd(vscale(X, v.x), vscale(Y, v.y)), vscale(Z, v.z)); }
static v3 local_to_world_normal(v3 v, v3 n) {
    v3 dx0 = V(0.0f, n.z, -n.y), dx1 = V(-n.z, 0.0f, n.x);
    v3 s = normalize(n.y * n.y > n.x * n.x ? dx0 : dx1);
    v3 t = normalize(cross(n, s));
    return local_to_world(v, s, t, n);
}

/* KIRK::Ray (Common/Ray.cpp:11-26): direction normalised at construction */
typedef struct { v3 o, d; } ray_t;
static ray_t make_ray(v3 o, v3 d) { ray_t r; r.o = o; r.d = normalize(d); return r; }
static v3 follow(const ray_t* r, float t) { return vadd(vscale(r->d, t), r->o); }

/* ======================================================================= */
/*  objects: Triangle and Cylinder constructors                             */
/* ======================================================================= */
#define RAY_EPS 1e-4f          /* KIRK::cRayEpsilon, Common/Ray.h:9   */
#define TRI_EPS 1e-7f          /* cTriangleEpsilon, Common/Triangle.h:46 */

typedef struct {
    int is_cone;
    v3 bmin, bmax, centroid;
    uint32_t mat;
    /* triangle */
    v3 A, B, C, ab, ac, bc, na, nb, nc, nrm;
    int lA;
    /* cone */
    v3 base, apex, u, v, w;
    float r0, r1, height, slope, base_d, min_d, max_d;
    /* texcoords m_tca, m_tcb, m_tcc after the ctor's vertex reordering (triangles) */
    float tc[6];
} obj_t;

/* Triangle::Triangle (Common/Triangle.cpp:3-129), identity model matrix.  The
 * texcoords tca/tcb/tcc (uv: 6 floats or NULL) follow the vertex reordering. */
static void tri_ctor(obj_t* o, v3 a, v3 b, v3 c, v3 na, v3 nb, v3 nc, const float* uv) {
    memset(o, 0, sizeof(*o));
    o->bmin = vsub(v3min(v3min(a, b), c), V(RAY_EPS, RAY_EPS, RAY_EPS));
    o->bmax = vadd(v3max(v3max(a, b), c), V(RAY_EPS, RAY_EPS, RAY_EPS));
    v3 diff = vsub(o->bmax, o->bmin);
    int lA = 0;
    float longest = diff.x;
    if (diff.y > longest) { longest = diff.y; lA = 1; }
    if (diff.z > longest) { longest = diff.z; lA = 2; }
    o->lA = lA;
    v3 Na = normalize(na), Nb = normalize(nb), Nc = normalize(nc);
    o->A = a; o->B = b; o->C = c; o->na = Na; o->nb = Nb; o->nc = Nc;
    float ca = comp(a, lA), cb = comp(b, lA), cc = comp(c, lA);
    static const float zero_uv[6] = {0, 0, 0, 0, 0, 0};
    const float* t = uv ? uv : zero_uv;
    float ta[2] = {t[0], t[1]}, tb[2] = {t[2], t[3]}, tcc[2] = {t[4], t[5]};
    const float *TA = ta, *TB = tb, *TC = tcc;
    if (ca <= cb && cb <= cc) { o->A = a; o->B = b; o->C = c; o->na = Na; o->nb = Nb; o->nc = Nc; TA = ta; TB = tb; TC = tcc; }
    if (cb <= ca && ca <= cc) { o->A = b; o->B = a; o->C = c; o->na = Nb; o->nb = Na; o->nc = Nc; TA = tb; TB = ta; TC = tcc; }
    if (ca <= cc && cc <= cb) { o->A = a; o->B = c; o->C = b; o->na = Na; o->nb = Nc; o->nc = Nb; TA = ta; TB = tcc; TC = tb; }
    if (cc <= ca && ca <= cb) { o->A = c; o->B = a; o->C = b; o->na = Nc; o->nb = Na; o->nc = Nb; TA = tcc; TB = ta; TC = tb; }
    if (cb <= cc && cc <= ca) { o->A = b; o->B = c; o->C = a; o->na = Nb; o->nb = Nc; o->nc = Na; TA = tb; TB = tcc; TC = ta; }
    if (cc <= cb && cb <= ca) { o->A = c; o->B = b; o->C = a; o->na = Nc; o->nb = Nb; o->nc = Na; TA = tcc; TB = tb; TC = ta; }
    o->tc[0] = TA[0]; o->tc[1] = TA[1]; o->tc[2] = TB[0]; o->tc[3] = TB[1]; o->tc[4] = TC[0]; o->tc[5] = TC[1];
    o->ab = vsub(o->B, o->A);
    o->ac = vsub(o->C, o->A);
    o->bc = vsub(o->C, o->B);
    if (comp(o->ab, lA) == 0.0f) set_comp(&o->ab, lA, 0.0001f);
    if (comp(o->ac, lA) == 0.0f) set_comp(&o->ac, lA, 0.0001f);
    if (comp(o->bc, lA) == 0.0f) set_comp(&o->bc, lA, 0.0001f);
    o->nrm = normalize(vdivs(vadd(vadd(o->na, o->nb), o->nc), 3.0f));
    o->centroid = vdivs(vadd(vadd(o->A, o->B), o->C), 3.0f);
}

/* glm 0.9.9 (func_matrix.inl compute_inverse<4,4>): Coef/Fac/Vec/Inv with
 * SignA = (+,-,+,-), SignB = (-,+,-,+), determinant = (d0 + d1) + (d2 + d3)
 * over the first column of M and the first row of the adjugate; returns
 * mat3(transpose(inverse(M))) column-major in ti.  M column-major, M[4c+r]. */
static void glm_inverse_transpose3(const float* M, float* ti) {
    float m[4][4];
    for (int cc = 0; cc < 4; ++cc) for (int r = 0; r < 4; ++r) m[cc][r] = M[4 * cc + r];
    float Coef00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
    float Coef02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float Coef03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float Coef04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float Coef06 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float Coef07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float Coef08 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
    float Coef10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float Coef11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float Coef12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float Coef14 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float Coef15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float Coef16 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
    float Coef18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float Coef19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float Coef20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float Coef22 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
    float Coef23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    float Fac0[4] = {Coef00, Coef00, Coef02, Coef03}, Fac1[4] = {Coef04, Coef04, Coef06, Coef07};
    float Fac2[4] = {Coef08, Coef08, Coef10, Coef11}, Fac3[4] = {Coef12, Coef12, Coef14, Coef15};
    float Fac4[4] = {Coef16, Coef16, Coef18, Coef19}, Fac5[4] = {Coef20, Coef20, Coef22, Coef23};
    float Vec0[4] = {m[1][0], m[0][0], m[0][0], m[0][0]}, Vec1[4] = {m[1][1], m[0][1], m[0][1], m[0][1]};
    float Vec2[4] = {m[1][2], m[0][2], m[0][2], m[0][2]}, Vec3[4] = {m[1][3], m[0][3], m[0][3], m[0][3]};
    const float SignA[4] = {1.0f, -1.0f, 1.0f, -1.0f}, SignB[4] = {-1.0f, 1.0f, -1.0f, 1.0f};
    float inv[4][4];
    for (int i = 0; i < 4; ++i) {
        inv[0][i] = ((Vec1[i] * Fac0[i] - Vec2[i] * Fac1[i]) + Vec3[i] * Fac2[i]) * SignA[i];
        inv[1][i] = ((Vec0[i] * Fac0[i] - Vec2[i] * Fac3[i]) + Vec3[i] * Fac4[i]) * SignB[i];
        inv[2][i] = ((Vec0[i] * Fac1[i] - Vec1[i] * Fac3[i]) + Vec3[i] * Fac5[i]) * SignA[i];
        inv[3][i] = ((Vec0[i] * Fac2[i] - Vec1[i] * Fac4[i]) + Vec2[i] * Fac5[i]) * SignB[i];
    }
    float Dot0[4] = {m[0][0] * inv[0][0], m[0][1] * inv[1][0], m[0][2] * inv[2][0], m[0][3] * inv[3][0]};
    float Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3]);
    float OneOverDeterminant = 1.0f / Dot1;
    for (int cc = 0; cc < 3; ++cc) for (int r = 0; r < 3; ++r) ti[3 * cc + r] = inv[r][cc] * OneOverDeterminant;
}
/* vec3(M * vec4(p, w)), glm's ((m0 x + m1 y) + (m2 z + m3 w)) */
static v3 glm_m4v(const float* M, v3 p, float w) {
    return V((M[0] * p.x + M[4] * p.y) + (M[8] * p.z + M[12] * w), (M[1] * p.x + M[5] * p.y) + (M[9] * p.z + M[13] * w),
             (M[2] * p.x + M[6] * p.y) + (M[10] * p.z + M[14] * w));
}
/* mat3 * vec3, glm's (m[0] x + m[1] y) + m[2] z per row */
static v3 glm_m3v(const float* A, v3 p) {
    return V((A[0] * p.x + A[3] * p.y) + A[6] * p.z, (A[1] * p.x + A[4] * p.y) + A[7] * p.z,
             (A[2] * p.x + A[5] * p.y) + A[8] * p.z);
}

/* Cylinder::Cylinder + computeBounds (Common/Cylinder.cpp:5-67, 306-336).  M:
 * the node transform (glm::mat4, column-major) or NULL for world-space cones
 * (then the matrix products are skipped: identity up to the sign of zeros).
 * Frame and height from the PRE-transform points (Cylinder.cpp:17-25), frame
 * mapped by mat3(transpose(inverse(M))) (:26-29), base/apex by M (:8-9). */
static void cone_ctor(obj_t* o, v3 base_in, v3 apex_in, float r0, float r1, const float* M) {
    memset(o, 0, sizeof(*o));
    o->is_cone = 1;
    v3 base = base_in, apex = apex_in;
    if (M) { base = glm_m4v(M, base_in, 1.0f); apex = glm_m4v(M, apex_in, 1.0f); }
    o->base = base; o->apex = apex; o->r0 = r0; o->r1 = r1;
    v3 v = vsub(apex_in, base_in);
    o->height = length(v);
    v = normalize(v);
    v3 tmp = V(0.0f, 1.0f, 0.0f);
    if (1.0f - fabsf(dot(tmp, v)) < RAY_EPS) tmp = V(0.0f, 0.0f, 1.0f);
    v3 u = normalize(cross(v, tmp));
    v3 w = normalize(cross(u, v));
    if (M) {
        float ti[9];
        glm_inverse_transpose3(M, ti);
        u = glm_m3v(ti, u); v = glm_m3v(ti, v); w = glm_m3v(ti, w);
    }
    o->u = normalize(u); o->v = normalize(v); o->w = normalize(w);
    o->slope = (r0 - r1) / o->height;
    o->base_d = dot(base, o->v);
    o->min_d = dot(o->v, base);
    o->max_d = dot(o->v, apex);
    if (o->max_d < o->min_d) { float t = o->max_d; o->max_d = o->min_d; o->min_d = t; }
    /* computeBounds */
    float radius = (r0 > r1) ? r0 + 1e-6f : r1 + 1e-6f;
    v3 l0 = V(-radius, 0.0f, -radius), l1 = V(radius, o->height, radius);
    v3 corners[8] = {V(l0.x, l1.y, l1.z), V(l0.x, l0.y, l1.z), V(l1.x, l0.y, l1.z), V(l1.x, l1.y, l1.z),
                     V(l1.x, l1.y, l0.z), V(l1.x, l0.y, l0.z), V(l0.x, l0.y, l0.z), V(l0.x, l1.y, l0.z)};
    o->bmin = V(FLT_MAX, FLT_MAX, FLT_MAX);
    o->bmax = V(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (int i = 0; i < 8; ++i) {
        v3 q = corners[i];
        /* mat3(u,v,w) * q + base */
        v3 P = V((o->u.x * q.x + o->v.x * q.y) + o->w.x * q.z, (o->u.y * q.x + o->v.y * q.y) + o->w.y * q.z,
                 (o->u.z * q.x + o->v.z * q.y) + o->w.z * q.z);
        P = vadd(P, base);
        if (P.x < o->bmin.x) o->bmin.x = P.x;
        if (P.x > o->bmax.x) o->bmax.x = P.x;
        if (P.y < o->bmin.y) o->bmin.y = P.y;
        if (P.y > o->bmax.y) o->bmax.y = P.y;
        if (P.z < o->bmin.z) o->bmin.z = P.z;
        if (P.z > o->bmax.z) o->bmax.z = P.z;
    }
    /* m_centroid = m_basepoint + 0.4 * (apexPoint - basePoint): transformed base,
     * pre-transform axis (Cylinder.cpp:50) */
    o->centroid = vadd(base, vscale(vsub(apex_in, base_in), 0.4f));
}

/* Intersection record (Common/Intersection.cpp:12-28) */
typedef struct {
    float lambda;
    int obj;
    float bu, bv;     /* barycentric u,v (triangles); 0 for cones */
} hit_t;

/* Triangle::closestIntersection (Triangle.cpp:152-184) */
static int tri_closest(const obj_t* o, const ray_t* r, hit_t* h, int id, float tMin, float tMax) {
    v3 dv = cross(r->d, o->ac);
    float det = dot(dv, o->ab);
    if (fabsf(det) < TRI_EPS) return 0;
    float inv = 1.0f / det;
    v3 w = vsub(r->o, o->A);
    float u = dot(dv, w) * inv;
    if (u < 0.0f || u > 1.0f) return 0;
    v3 wu = cross(w, o->ab);
    float v = dot(wu, r->d) * inv;
    if (v < 0.0f || u + v > 1.0f) return 0;
    float t = dot(wu, o->ac) * inv;
    if ((t < tMin) || (t > tMax)) return 0;
    h->lambda = t; h->obj = id; h->bu = u; h->bv = v;
    return 1;
}
/* Triangle::isIntersection (Triangle.cpp:213-242) */
static int tri_any(const obj_t* o, const ray_t* r, float tMax) {
    v3 dv = cross(r->d, o->ac);
    float det = dot(dv, o->ab);
    if (fabsf(det) < TRI_EPS) return 0;
    float inv = 1.0f / det;
    v3 w = vsub(r->o, o->A);
    float u = dot(dv, w) * inv;
    if (u < 0.0f || u > 1.0f) return 0;
    v3 wu = cross(w, o->ab);
    float v = dot(wu, r->d) * inv;
    if (v < 0.0f || u + v > 1.0f) return 0;
    float t = dot(wu, o->ac) * inv;
    if ((t < 0.0f) || (t > tMax)) return 0;
    return 1;
}

/* Cylinder::closestIntersection (Cylinder.cpp:73-156): open cone frustum. */
static int cone_closest(const obj_t* o, const ray_t* r, hit_t* h, int id, float tMin, float tMax) {
    v3 P = vsub(r->o, o->base);
    v3 dir = r->d;
    P = V(dot(P, o->u), dot(P, o->v), dot(P, o->w));
    v3 D = V(dot(dir, o->u), dot(dir, o->v), dot(dir, o->w));
    float a = 1.0f - D.y * D.y * (1.0f + o->slope * o->slope);
    float b = P.x * D.x + P.z * D.z + o->r0 * o->slope * D.y - o->slope * o->slope * P.y * D.y;
    float c = o->r0 - o->slope * P.y;
    c = P.x * P.x + P.z * P.z - c * c;
    float disc = b * b - a * c;
    if (disc < 0.0f) return 0;
    disc = sqrtf(disc);
    float t1 = (-b - disc) / a;
    float t2 = (-b + disc) / a;
    if ((t2 < tMin) || (t1 > tMax)) return 0;
    if (t1 < RAY_EPS) {
        if ((t2 > tMax) || (t2 < tMin)) return 0;
        float d = dot(o->v, follow(r, t2));
        if (d >= o->min_d && d <= o->max_d) { h->lambda = t2; h->obj = id; h->bu = 0.0f; h->bv = 0.0f; return 1; }
        return 0;
    }
    if ((t1 < tMin) && (t2 > tMax)) return 0;
    float d = dot(o->v, follow(r, t1));
    if (d >= o->min_d && d <= o->max_d) { h->lambda = t1; h->obj = id; h->bu = 0.0f; h->bv = 0.0f; return 1; }
    d = dot(o->v, follow(r, t2));
    if (d >= o->min_d && d <= o->max_d) { h->lambda = t2; h->obj = id; h->bu = 0.0f; h->bv = 0.0f; return 1; }
    return 0;
}
/* Cylinder::isIntersection (Cylinder.cpp:158-228): note the different `a`. */
static int cone_any(const obj_t* o, const ray_t* r, float tMax) {
    v3 P = vsub(r->o, o->base);
    v3 dir = r->d;
    P = V(dot(P, o->u), dot(P, o->v), dot(P, o->w));
    v3 D = V(dot(dir, o->u), dot(dir, o->v), dot(dir, o->w));
    float a = D.x * D.x + D.z * D.z - o->slope * o->slope * D.y * D.y;
    float b = P.x * D.x + P.z * D.z + o->r0 * o->slope * D.y - o->slope * o->slope * P.y * D.y;
    float c = o->r0 - o->slope * P.y;
    c = P.x * P.x + P.z * P.z - c * c;
    float disc = b * b - a * c;
    if (disc < 0.0f) return 0;
    disc = sqrtf(disc);
    float t1 = (-b - disc) / a;
    float t2 = (-b + disc) / a;
    if ((t2 < 0.0f) || (t1 > tMax)) return 0;
    if (t1 < RAY_EPS) {
        if ((t2 > tMax) || (t2 < 0.0f)) return 0;
        float d = dot(o->v, follow(r, t2));
        return (d >= o->min_d && d <= o->max_d);
    }
    if ((t1 < 0.0f) && (t2 > tMax)) return 0;
    float d = dot(o->v, follow(r, t1));
    if (d >= o->min_d && d <= o->max_d) return 1;
    d = dot(o->v, follow(r, t2));
    return (d >= o->min_d && d <= o->max_d);
}

/* calcNormal: Cylinder.cpp:230-237, Triangle.cpp:244-248 */
static v3 obj_normal(const obj_t* o, const ray_t* r, const hit_t* h) {
    if (o->is_cone) {
        v3 Q = follow(r, h->lambda);
        float t = dot(Q, o->v) - o->base_d;
        v3 q1 = vsub(Q, vscale(o->v, t));
        v3 n = normalize(vsub(q1, o->base));
        return normalize(vadd(n, vscale(o->v, o->slope)));
    }
    float bx = (1.0f - h->bu) - h->bv;
    return normalize(vadd(vadd(vscale(o->na, bx), vscale(o->nb, h->bu)), vscale(o->nc, h->bv)));
}

/* ======================================================================= */
/*  BVH: BoundingBox + BVHNode::split/partition/traverse (CPU_BVH.cpp)      */
/* ======================================================================= */
typedef struct { v3 mn, mx; } box_t;
static box_t box_empty(void) {   /* BoundingBox() (BoundingBox.cpp:8-12) */
    box_t b; b.mn = V(FLT_MAX, FLT_MAX, FLT_MAX); b.mx = V(-FLT_MAX, -FLT_MAX, -FLT_MAX); return b;
}
static float smin(float a, float b) { return (b < a) ? b : a; }   /* std::min */
static float smax(float a, float b) { return (a < b) ? b : a; }   /* std::max */
static void box_grow_pt(box_t* b, v3 p) {
    b->mn = V(smin(b->mn.x, p.x), smin(b->mn.y, p.y), smin(b->mn.z, p.z));
    b->mx = V(smax(b->mx.x, p.x), smax(b->mx.y, p.y), smax(b->mx.z, p.z));
}
static void box_grow_box(box_t* b, const box_t* o) {
    b->mn = V(smin(b->mn.x, o->mn.x), smin(b->mn.y, o->mn.y), smin(b->mn.z, o->mn.z));
    b->mx = V(smax(b->mx.x, o->mx.x), smax(b->mx.y, o->mx.y), smax(b->mx.z, o->mx.z));
}
static float box_area(const box_t* b) {   /* BoundingBox::surfaceArea (BoundingBox.cpp:95-100) */
    v3 s = vsub(b->mx, b->mn);
    return 2.0f * (s.x * s.y + s.x * s.z + s.y * s.z);
}
static int box_worth(const box_t* b) {     /* worthSplitting (BoundingBox.cpp:102-107) */
    v3 d = vsub(b->mx, b->mn);
    return d.x > 0.0f && d.y > 0.0f && d.z > 0.0f;
}
/* BoundingVolume::intersects (BoundingBox.cpp:142-194) */
static int box_hit(const box_t* b, const ray_t* r, v3 inv, const int sgn[3], float* tmin_o, float* tmax_o) {
    const v3* bb = &b->mn;   /* bb[0]=mn, bb[1]=mx */
    v3 B0 = sgn[0] ? b->mx : b->mn, B1 = sgn[0] ? b->mn : b->mx;
    float tmin = (B0.x - r->o.x) * inv.x;
    float tmax = (B1.x - r->o.x) * inv.x;
    B0 = sgn[1] ? b->mx : b->mn; B1 = sgn[1] ? b->mn : b->mx;
    float tymin = (B0.y - r->o.y) * inv.y;
    float tymax = (B1.y - r->o.y) * inv.y;
    (void)bb;
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    B0 = sgn[2] ? b->mx : b->mn; B1 = sgn[2] ? b->mn : b->mx;
    float tzmin = (B0.z - r->o.z) * inv.z;
    float tzmax = (B1.z - r->o.z) * inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    *tmin_o = tmin; *tmax_o = tmax;
    return 1;
}

typedef struct {
    box_t box;
    int32_t left, right;      /* children (interior) */
    int32_t first, count;     /* leaf candidate range into object_ids; count 0 = interior */
} node_t;

typedef struct {
    uint32_t w, h, ch, wrap;
    uint8_t* data;
} tex_t;

struct ko_ctx {
    uint32_t n_obj, n_tris, n_cones;
    obj_t* obj;
    khp_material* mats; uint32_t n_mats;
    /* textures (ABI 6): KIRK::Texture, per-material texture indices, environment map */
    tex_t* tex; uint32_t n_tex;
    khp_material_textures* mtex;   /* NULL: untextured */
    khp_env_map env_map;
    int textured;
    struct ko_light* lights; uint32_t n_lights;
    khp_environment env;
    khp_camera cam;
    node_t* nodes; uint32_t n_nodes, cap_nodes, depth;
    uint32_t* ids;
    /* light-path variant (ABI 7): parameters and the subpaths of
     * the sample indices of the current render call */
    khp_bdpt_params bd;
    struct lvert* lv; size_t lv_cap;
    uint32_t lv_k0, lv_nk;
};

typedef struct { float cbmin, k; } axis_const_t;

static int32_t new_node(struct ko_ctx* c) {
    if (c->n_nodes == c->cap_nodes) {
        c->cap_nodes = c->cap_nodes ? c->cap_nodes * 2 : 1024;
        c->nodes = (node_t*)realloc(c->nodes, sizeof(node_t) * c->cap_nodes);
    }
    memset(&c->nodes[c->n_nodes], 0, sizeof(node_t));
    return (int32_t)c->n_nodes++;
}

static float cent(const struct ko_ctx* c, uint32_t id, int axis) { return comp(c->obj[id].centroid, axis); }

/* BVHNode::partition, binned SAH (CPU_BVH.cpp:357-552) */
static void partition(struct ko_ctx* c, uint32_t first, uint32_t second, uint32_t* lr_second, uint32_t* rr_first,
                      const box_t* centbox, box_t* lcb, box_t* rcb) {
    uint32_t* ids = c->ids;
    float best = FLT_MAX;
    int best_axis = 0, best_plane = 0;
    enum { NB = 16, NP = 15 };
    axis_const_t ac[3];
    for (int axis = 0; axis < 3; ++axis) {
        const float cbmin = comp(centbox->mn, axis);
        const float cbmax = comp(centbox->mx, axis);
        const float cbdiff = cbmax - cbmin;
        const float epsilon = 0.1f;
        const float k = ((float)NB * (1.0f - epsilon)) / cbdiff;
        ac[axis].cbmin = cbmin; ac[axis].k = k;
        box_t bin_b[NB]; uint32_t bin_n[NB];
        for (int i = 0; i < NB; ++i) { bin_b[i] = box_empty(); bin_n[i] = 0; }
        for (uint32_t id = first; id <= second; ++id) {
            uint32_t oid = ids[id];
            int bin = (int)(k * (cent(c, oid, axis) - cbmin));
            box_grow_pt(&bin_b[bin], c->obj[oid].centroid);
            ++bin_n[bin];
        }
        uint32_t left_n[NP]; box_t left_b[NP];
        left_b[0] = box_empty(); box_grow_box(&left_b[0], &bin_b[0]);
        left_n[0] = bin_n[0];
        for (int p = 1; p < NP; ++p) {
            left_b[p] = box_empty();
            box_grow_box(&left_b[p], &left_b[p - 1]);
            box_grow_box(&left_b[p], &bin_b[p]);
            left_n[p] = left_n[p - 1] + bin_n[p];
        }
        uint32_t right_n[NP]; box_t right_b[NP];
        for (int p = NP - 1; p >= 0; --p) {
            right_b[p] = box_empty();
            box_grow_box(&right_b[p], &bin_b[p + 1]);
            right_n[p] = bin_n[p + 1];
            if (p != NP - 1) {
                box_grow_box(&right_b[p], &right_b[p + 1]);
                right_n[p] += right_n[p + 1];
            }
            float sal = box_area(&left_b[p]);
            float sar = box_area(&right_b[p]);
            float cost = sal * (float)left_n[p] + sar * (float)right_n[p];
            if (cost < best) {
                best = cost; best_axis = axis; best_plane = p;
                *lcb = left_b[p]; *rcb = right_b[p];
            }
        }
    }
    const float cbmin = ac[best_axis].cbmin, k = ac[best_axis].k;
    int left = (int)first, right = (int)second;
    int ls = 0, rs = 0;
    while (left < right) {
        if (!ls) {
            int b = (int)(k * (cent(c, ids[left], best_axis) - cbmin));
            if (b > best_plane) ls = 1; else ++left;
        }
        if (!rs) {
            int b = (int)(k * (cent(c, ids[right], best_axis) - cbmin));
            if (b <= best_plane) rs = 1; else --right;
        }
        if (ls && rs) {
            uint32_t t = ids[left]; ids[left] = ids[right]; ids[right] = t;
            ls = 0; rs = 0; ++left; --right;
        }
    }
    if (left > right) { *lr_second = (uint32_t)right; *rr_first = (uint32_t)left; }
    else if (ls) { *lr_second = (uint32_t)(left - 1); *rr_first = (uint32_t)left; }
    else if (rs) { *lr_second = (uint32_t)right; *rr_first = (uint32_t)(right + 1); }
    else {
        int b = (int)(k * (cent(c, ids[left], best_axis) - cbmin));
        if (b > best_plane) { *lr_second = (uint32_t)(left - 1); *rr_first = (uint32_t)left; }
        else { *lr_second = (uint32_t)left; *rr_first = (uint32_t)(left + 1); }
    }
}

/* BVHNode::split (CPU_BVH.cpp:95-138), leaf_threshold 1, unbounded depth (CPU_BVH.h:64) */
static int32_t split(struct ko_ctx* c, uint32_t first, uint32_t second, const box_t* centbox, uint32_t depth) {
    int32_t ni = new_node(c);
    box_t bv = box_empty();   /* computeBoundaries (BoundingBox.cpp:117-140) */
    for (uint32_t id = first; id <= second; ++id) {
        const obj_t* o = &c->obj[c->ids[id]];
        bv.mn = V(smin(bv.mn.x, o->bmin.x), smin(bv.mn.y, o->bmin.y), smin(bv.mn.z, o->bmin.z));
        bv.mx = V(smax(bv.mx.x, o->bmax.x), smax(bv.mx.y, o->bmax.y), smax(bv.mx.z, o->bmax.z));
    }
    c->nodes[ni].box = bv;
    if (depth > c->depth) c->depth = depth;
    if (second - first > 1u && box_worth(centbox)) {
        uint32_t ls, rf;
        box_t lcb, rcb;
        partition(c, first, second, &ls, &rf, centbox, &lcb, &rcb);
        int32_t l = split(c, first, ls, &lcb, depth + 1);
        int32_t r = split(c, rf, second, &rcb, depth + 1);
        c->nodes[ni].left = l; c->nodes[ni].right = r; c->nodes[ni].count = 0;
    } else {
        c->nodes[ni].first = (int32_t)first;
        c->nodes[ni].count = (int32_t)(second - first + 1);
        c->nodes[ni].left = c->nodes[ni].right = -1;
    }
    return ni;
}

/* --- traversal ------------------------------------------------------------ */
typedef struct {
    uint64_t nodes, prims;
    int32_t* log;        /* optional visit log (tools/treelet_sim.py): preorder ids of visited nodes, */
    uint64_t log_n, log_cap;   /* with bits 25..31 = deferred far children at the visit (min 127) */
    int32_t pending;
} trav_stats_t;

/* BVHNode::traverse(Intersection*) (CPU_BVH.cpp:148-199) + Container::closestIntersectionWithCandidates
 * (Container.cpp:13-25). */
static void trav_closest(const struct ko_ctx* c, int32_t ni, const ray_t* r, v3 inv, const int sgn[3], float tmin,
                         float tmax, hit_t* hit, trav_stats_t* st) {
    if (tmax < 0.0f || tmin > hit->lambda) return;
    const node_t* n = &c->nodes[ni];
    if (st) {
        st->nodes++;
        if (st->log && st->log_n < st->log_cap)
            st->log[st->log_n] = ni | ((st->pending < 127 ? st->pending : 127) << 25);
        if (st->log) st->log_n++;
    }
    if (n->count > 0) {
        hit_t tmp; tmp.lambda = FLT_MAX; tmp.obj = -1; tmp.bu = tmp.bv = 0.0f;
        int found = 0;
        float tMax = tmax;
        for (int32_t k = 0; k < n->count; ++k) {
            uint32_t id = c->ids[n->first + k];
            const obj_t* o = &c->obj[id];
            if (st) st->prims++;
            int ok = o->is_cone ? cone_closest(o, r, &tmp, (int)id, 0.0f, tMax) : tri_closest(o, r, &tmp, (int)id, 0.0f, tMax);
            if (ok) { tMax = tmp.lambda; found = 1; }
        }
        if (found && tmp.lambda < hit->lambda) *hit = tmp;
        return;
    }
    float lt0, lt1, rt0, rt1;
    int lh = box_hit(&c->nodes[n->left].box, r, inv, sgn, &lt0, &lt1);
    int rh = box_hit(&c->nodes[n->right].box, r, inv, sgn, &rt0, &rt1);
    if (lh && rh) {
        if (st) st->pending++;   /* the far child waits while the near one is traversed */
        if (lt0 < rt0) {
            trav_closest(c, n->left, r, inv, sgn, lt0, lt1, hit, st);
            if (st) st->pending--;
            trav_closest(c, n->right, r, inv, sgn, rt0, rt1, hit, st);
        } else {
            trav_closest(c, n->right, r, inv, sgn, rt0, rt1, hit, st);
            if (st) st->pending--;
            trav_closest(c, n->left, r, inv, sgn, lt0, lt1, hit, st);
        }
    } else if (lh) {
        trav_closest(c, n->left, r, inv, sgn, lt0, lt1, hit, st);
    } else if (rh) {
        trav_closest(c, n->right, r, inv, sgn, rt0, rt1, hit, st);
    }
}

/* BVHNode::traverse(Ray*) (CPU_BVH.cpp:211-265) + isIntersectionWithCandidates (Container.cpp:27-34) */
static int trav_any(const struct ko_ctx* c, int32_t ni, const ray_t* r, v3 inv, const int sgn[3], float tmin,
                    float tmax, float tMax, trav_stats_t* st) {
    if (tmax < 0.0f || tmin > tMax) return 0;
    const node_t* n = &c->nodes[ni];
    if (st) st->nodes++;
    if (n->count > 0) {
        for (int32_t k = 0; k < n->count; ++k) {
            const obj_t* o = &c->obj[c->ids[n->first + k]];
            if (st) st->prims++;
            if (o->is_cone ? cone_any(o, r, tMax) : tri_any(o, r, tMax)) return 1;
        }
        return 0;
    }
    float lt0, lt1, rt0, rt1;
    int lh = box_hit(&c->nodes[n->left].box, r, inv, sgn, &lt0, &lt1);
    int rh = box_hit(&c->nodes[n->right].box, r, inv, sgn, &rt0, &rt1);
    if (lh && rh) {
        if (lt0 < rt0) {
            if (trav_any(c, n->left, r, inv, sgn, lt0, lt1, tMax, st)) return 1;
            if (trav_any(c, n->right, r, inv, sgn, rt0, rt1, tMax, st)) return 1;
        } else {
            if (trav_any(c, n->right, r, inv, sgn, rt0, rt1, tMax, st)) return 1;
            if (trav_any(c, n->left, r, inv, sgn, lt0, lt1, tMax, st)) return 1;
        }
    } else if (lh) {
        if (trav_any(c, n->left, r, inv, sgn, lt0, lt1, tMax, st)) return 1;
    } else if (rh) {
        if (trav_any(c, n->right, r, inv, sgn, rt0, rt1, tMax, st)) return 1;
    }
    return 0;
}

static v3 inv_dir(v3 d, int sgn[3]) {
    sgn[0] = d.x < 0.0f; sgn[1] = d.y < 0.0f; sgn[2] = d.z < 0.0f;
    return V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
}

/* BVH::closestIntersection (CPU_BVH.cpp:51-69) */
static int bvh_closest(const struct ko_ctx* c, const ray_t* r, hit_t* hit, trav_stats_t* st) {
    hit->lambda = FLT_MAX; hit->obj = -1; hit->bu = hit->bv = 0.0f;
    if (c->n_nodes == 0) return 0;
    int sgn[3];
    v3 inv = inv_dir(r->d, sgn);
    float tmin, tmax;
    if (!box_hit(&c->nodes[0].box, r, inv, sgn, &tmin, &tmax)) return 0;
    trav_closest(c, 0, r, inv, sgn, tmin, tmax, hit, st);
    return hit->obj >= 0;
}
/* BVH::isIntersection (CPU_BVH.cpp:77-93) */
static int bvh_any(const struct ko_ctx* c, const ray_t* r, float tMax, trav_stats_t* st) {
    if (c->n_nodes == 0) return 0;
    int sgn[3];
    v3 inv = inv_dir(r->d, sgn);
    float tmin, tmax;
    if (!box_hit(&c->nodes[0].box, r, inv, sgn, &tmin, &tmax)) return 0;
    return trav_any(c, 0, r, inv, sgn, tmin, tmax, tMax, st);
}

/* ======================================================================= */
/*  lights (Common/Light.h, Common/Light.cpp)                               */
/* ======================================================================= */
struct ko_light {
    int kind;
    v3 color, position, direction;
    float radius, c, l, q, inner, outer;
    v3 vert[4];
};
typedef struct ko_light light_t;

/* Light::orthonormalBase (Light.cpp:112-118) */
static void ortho_base(v3 n, v3* s, v3* t) {
    *s = fabsf(n.x) > fabsf(n.y) ? vdivs(V(-n.z, 0.0f, n.x), sqrtf(n.x * n.x + n.z * n.z))
                                 : vdivs(V(0.0f, n.z, -n.y), sqrtf(n.y * n.y + n.z * n.z));
    *t = cross(n, *s);
}

/* ctor + QuadLight::calcParams + Light::transform(identity) (Light.h ctor, Light.cpp:216-220, 263-276) */
static void light_init(light_t* L, const khp_light* in) {
    memset(L, 0, sizeof(*L));
    L->kind = in->kind;
    L->color = ld3(in->color);
    L->position = ld3(in->position);
    L->c = in->att_const; L->l = in->att_lin; L->q = in->att_quad;
    L->radius = in->radius;
    v3 dir1 = normalize(ld3(in->direction));
    if (in->kind == KHP_LIGHT_POINT) dir1 = normalize(V(0.0f, 0.0f, 0.0f));
    if (in->kind == KHP_LIGHT_SPOT) {
        L->outer = in->outer_angle;
        L->inner = (in->inner_angle < 0.0f || in->inner_angle > in->outer_angle) ? in->outer_angle : in->inner_angle;
    }
    if (in->kind == KHP_LIGHT_QUAD) {
        v3 s, t;
        ortho_base(dir1, &s, &t);
        float sx = in->size[0], sy = in->size[1];
        L->vert[0] = vadd(vadd(L->position, vdivs(vscale(s, -sx), 2.0f)), vdivs(vscale(t, -sy), 2.0f));
        L->vert[1] = vadd(vadd(L->position, vdivs(vscale(s, sx), 2.0f)), vdivs(vscale(t, -sy), 2.0f));
        L->vert[2] = vadd(vadd(L->position, vdivs(vscale(s, sx), 2.0f)), vdivs(vscale(t, sy), 2.0f));
        L->vert[3] = vadd(vadd(L->position, vdivs(vscale(s, -sx), 2.0f)), vdivs(vscale(t, sy), 2.0f));
        L->radius = sqrtf((sx * sy) / K_PIF);
    }
    L->direction = normalize(dir1);   /* Light::transform re-normalises (Light.h transform) */
}

/* Light::distanceAttenuation (Light.h:70-73) */
static float dist_att(const light_t* L, float d) {
    return (L->c > 0.0f || (L->l > 0.0f && L->q > 0.0f)) ? 1.0f / ((L->c + L->l * d) + L->q * (d * d)) : 1.0f;
}

/* Light::uniformSampleSphere (Light.cpp:66-72): m_dist is a double distribution */
static v3 uniform_sphere(float u0, float u1) {
    float phi = (float)((double)u0 * 2.0 * K_M_PI);
    float ct = (float)(2.0 * (double)u1 - 1.0);
    float st = sqrtf(gmax(0.0f, 1.0f - ct * ct));
    return V(st * ko_cosf(phi), st * ko_sinf(phi), ct);
}

/* calcLightdir (Light.cpp:127-145, 278-296, 327-343, 463-475), randomize = true */
static ray_t light_dir(const light_t* L, v3 p, float u0, float u1, float* att) {
    if (L->kind == KHP_LIGHT_POINT) {
        v3 pos = L->position;
        v3 direction = normalize(vsub(pos, p));
        v3 pt = uniform_sphere(u0, u1);
        pos = vadd(pos, vscale(pt, L->radius));
        float dd = gclamp(dot(pt, vneg(direction)), 0.0f, 1.0f);
        float dist = length(vsub(pos, p));
        *att = dd * dist_att(L, dist);
        return make_ray(p, vsub(pos, p));
    }
    if (L->kind == KHP_LIGHT_QUAD) {
        float u = u0, v = u1;
        v3 x1 = vadd(L->vert[0], vscale(vsub(L->vert[1], L->vert[0]), u));
        v3 x2 = vadd(L->vert[3], vscale(vsub(L->vert[2], L->vert[3]), u));
        v3 ip = vadd(x1, vscale(vsub(x2, x1), v));
        v3 ld = vsub(ip, p);
        float dd = gclamp(dot(normalize(vneg(ld)), L->direction), 0.0f, 1.0f);
        *att = dd * dist_att(L, length(ld));
        return make_ray(p, ld);
    }
    if (L->kind == KHP_LIGHT_SPOT) {
        /* sampleDisk (Light.cpp:94-110) */
        float rr = sqrtf(u0);
        float th = (float)(2.0 * K_M_PI * (double)u1);
        float x = rr * ko_cosf(th), y = rr * ko_sinf(th);
        v3 d = V(L->radius * x, L->radius * y, 0.0f);
        v3 s, t;
        ortho_base(L->direction, &s, &t);
        v3 pt = vadd(vscale(s, d.x), vscale(t, d.y));
        v3 ld = vsub(vadd(L->position, pt), p);
        float ang = ko_acosf(dot(normalize(vneg(ld)), L->direction)) * K_RAD2DEG;
        float delta = 1.0f - gclamp((ang - L->inner) / (L->outer - L->inner), 0.0f, 1.0f);
        delta = delta * delta * delta * delta;
        *att = delta * dist_att(L, length(ld));
        return make_ray(p, ld);
    }
    /* sun */
    v3 pt = vscale(uniform_sphere(u0, u1), L->radius);
    pt = vsub(pt, L->direction);
    v3 dn = normalize(pt);
    v3 pos = vscale(dn, 1e16f);
    *att = 1.0f;
    return make_ray(p, vsub(pos, p));
}

/* Light::intersectTriangle (Light.cpp:13-64) */
static int light_tri(const ray_t* r, v3 v1, v3 v2, v3 v3_, float* t) {
    v3 e1 = vsub(v2, v1), e2 = vsub(v3_, v1);
    v3 P = cross(r->d, e2);
    float det = dot(e1, P);
    if (det > -FLT_EPSILON && det < FLT_EPSILON) return 0;
    float inv = 1.0f / det;
    v3 T = vsub(r->o, v1);
    float u = dot(T, P) * inv;
    if (u < 0.0f || u > 1.0f) return 0;
    v3 Q = cross(T, e1);
    float v = dot(r->d, Q) * inv;
    if (v < 0.0f || u + v > 1.0f) return 0;
    *t = dot(e2, Q) * inv;
    return *t > FLT_EPSILON;
}

/* isIntersection (Light.cpp:169-189, 227-232, 367-428, 497-501) */
static int light_isect(const light_t* L, const ray_t* r, float* t) {
    if (L->kind == KHP_LIGHT_POINT) {
        float rsq = L->radius * L->radius;
        if (rsq == 0.0f) return 0;
        if (dot(r->d, vsub(r->o, L->position)) > 0.0f) return 0;
        float a = dot(r->d, r->d);
        float b = dot(r->d, vscale(vsub(r->o, L->position), 2.0f));
        float c = ((dot(L->position, L->position) + dot(r->o, r->o)) - 2.0f * dot(r->o, L->position)) - rsq;
        float d = b * b - 4.0f * a * c;
        if (d < 0.0f) return 0;
        d = sqrtf(d);
        *t = (-0.5f) * (b + d) / a;
        return 1;
    }
    if (L->kind == KHP_LIGHT_QUAD) {
        return light_tri(r, L->vert[0], L->vert[1], L->vert[3], t) || light_tri(r, L->vert[2], L->vert[3], L->vert[1], t);
    }
    if (L->kind == KHP_LIGHT_SPOT) {
        if (L->radius == 0.0f) return 0;
        v3 n = L->direction;
        v3 x = fabsf(n.x) > fabsf(n.y) ? vdivs(V(-n.z, 0.0f, n.x), sqrtf(n.x * n.x + n.z * n.z))
                                       : vdivs(V(0.0f, n.z, -n.y), sqrtf(n.y * n.y + n.z * n.z));
        v3 y = cross(n, x);
        v3 v1 = L->position, v2 = vadd(L->position, x), v3_ = vadd(L->position, y);
        v3 e1 = vsub(v2, v1), e2 = vsub(v3_, v1);
        v3 P = cross(r->d, e2);
        float det = dot(e1, P);
        if (det > -FLT_EPSILON && det < FLT_EPSILON) return 0;
        float inv = 1.0f / det;
        v3 T = vsub(r->o, v1);
        float u = dot(T, P) * inv;
        v3 Q = cross(T, e1);
        float v = dot(r->d, Q) * inv;
        if (u * u + v * v > L->radius * L->radius) return 0;
        *t = dot(e2, Q) * inv;
        return *t > FLT_EPSILON;
    }
    return 0;   /* SunLight: never intersected */
}

/* sampleLightSource (Light.cpp:196-199, 234-239, 436-440, 508-511) */
static v3 light_emit(const light_t* L, v3 dir) {
    float cdiv = L->c > 0.0f ? L->c : 1.0f;
    if (L->kind == KHP_LIGHT_POINT) return vdivs(vscale(L->color, K_ONE_OVER_PI), cdiv);
    if (L->kind == KHP_LIGHT_QUAD || L->kind == KHP_LIGHT_SPOT) {
        float dd = dot(normalize(vneg(dir)), L->direction) < 0.0f ? 0.0f : 1.0f;
        return vdivs(vscale(L->color, K_ONE_OVER_PI * dd), cdiv);
    }
    return L->color;
}

/* ======================================================================= */
/*  BSDFs (Common/Shading/Bsdf.cpp)                                         */
/* ======================================================================= */
#define F_TRANSPARENT 1   /* BSDFHelper::MATFLAG_* (Bsdf.h:18-22) */
#define F_SPECULAR 2
#define F_EMISSIVE 4
#define F_CYL_T 8
#define F_CYL_TR 16

/* dialectricFresnel (Bsdf.cpp:143-171) */
static float fresnel_dielectric(float cos_theta, float eta_i, float eta_t) {
    float ci = gclamp(cos_theta, -1.0f, 1.0f);
    if (ci <= 0.0f) { float t = eta_i; eta_i = eta_t; eta_t = t; ci = fabsf(ci); }
    float si = sqrtf(gmax(0.0f, 1.0f - ci * ci));
    float st = eta_i / eta_t * si;
    if (st >= 1.0f) return 1.0f;
    float ct = sqrtf(gmax(0.0f, 1.0f - st * st));
    float rparl = ((eta_t * ci) - (eta_i * ct)) / ((eta_t * ci) + (eta_i * ct));
    float rperp = ((eta_i * ci) - (eta_t * ct)) / ((eta_i * ci) + (eta_t * ct));
    return (rparl * rparl + rperp * rperp) / 2.0f;
}
/* concentricSampleDisk / cosineSampleHemisphere / sampleAngle (Bsdf.cpp:95-132) */
static void concentric_disk(float u0, float u1, float* dx, float* dy) {
    float ox = 2.0f * u0 - 1.0f, oy = 2.0f * u1 - 1.0f;
    if (ox == 0.0f && oy == 0.0f) { *dx = 0.0f; *dy = 0.0f; return; }
    float th, r;
    if (fabsf(ox) > fabsf(oy)) { r = ox; th = K_QUARTER_PI * (oy / ox); }
    else { r = oy; th = K_HALF_PI - K_QUARTER_PI * (ox / oy); }
    *dx = r * ko_cosf(th); *dy = r * ko_sinf(th);
}
static v3 cosine_hemi(float u0, float u1) {
    float dx, dy;
    concentric_disk(u0, u1, &dx, &dy);
    return V(dx, dy, sqrtf(gmax(0.0f, 1.0f - dx * dx - dy * dy)));
}
static v3 sample_angle(float u0, float u1, float max_angle) {
    float phi = (float)((double)(u0 * 2.0f) * K_M_PI);
    float ct = 1.0f - u1 * (1.0f - ko_cosf(max_angle));
    float st = sqrtf(1.0f - ct * ct);
    return V(ko_cosf(phi) * st, ko_sinf(phi) * st, ct);
}
static float normal_gauss_pdf(float x, float mean, float sd) {   /* Bsdf.cpp:79-85 */
    const float inv_sqrt_2pi = 0.3989422804014327f;
    float a = (x - mean) / sd;
    return inv_sqrt_2pi / sd * ko_expf(-0.5f * a * a);
}

typedef struct {
    const obj_t* obj;
    const khp_material* m;
    v3 n;
} shade_ctx_t;

/* BSDF::evaluateLight dispatch */
static v3 bsdf_eval(const shade_ctx_t* s, v3 in, v3 out) {
    int kind = s->m->bsdf;
    if (kind == KHP_BSDF_LAMBERTIAN_REFLECTION || kind == KHP_BSDF_MARSCHNER_HAIR) {  /* Bsdf.cpp:197-202, 771-776 */
        if (dot(in, s->n) * dot(out, s->n) > 0.0f) return vscale(ld3(s->m->diffuse), K_ONE_OVER_PI);
        return V(0.0f, 0.0f, 0.0f);
    }
    if (kind == KHP_BSDF_LAMBERTIAN_TRANSMISSION) {   /* Bsdf.cpp:310-318 */
        if (!(dot(in, s->n) * dot(out, s->n) > 0.0f)) return vscale(ld3(s->m->diffuse), K_ONE_OVER_PI);
        return V(0.0f, 0.0f, 0.0f);
    }
    return V(0.0f, 0.0f, 0.0f);
}

/* Marschner R lobe (Bsdf.cpp:465-489, 669-736).  TT/TRT are unreachable: p = 0 is
 * hard-coded (:669) and no BSDF ever sets MATFLAG_CYLINDER_T/TR. */
static v3 marschner_r(const shade_ctx_t* s, v3 in, v3 n, float sample[2], const float hu[2], v3* out, float* pdf,
                      int* flags) {
    const obj_t* o = s->obj;
    v3 U = o->u, Vv = o->v, W = o->w;
    float ior = s->m->ior;
    v3 nin = normalize(in);
    v3 in_cyl = world_to_local(in, Vv, U, W);
    float alpha = -1.0f * (5.0f + 5.0f * hu[0]);
    float beta = 5.0f + 5.0f * hu[1];
    if ((*flags & F_CYL_T) || (*flags & F_CYL_TR)) { *out = V(0.0f, 0.0f, 1.0f); return V(0.0f, 0.0f, 0.0f); }
    v3 o1 = reflect(vneg(nin), faceforward(n, vneg(nin), n));
    o1 = rotate_rowvec(o1, alpha, Vv);
    *flags = F_SPECULAR;
    v3 oc = world_to_local(o1, Vv, U, W);
    float ti = ko_atan2f(k_hypotf(in_cyl.x, in_cyl.z), in_cyl.y);
    float tr = ko_atan2f(k_hypotf(oc.x, oc.z), oc.y);
    float th = (tr + ti) / 2.0f;
    float td = (tr - ti) / 2.0f;
    float gx = th - alpha;
    sample[0] = ti; sample[1] = 0.0f;
    *pdf = normal_gauss_pdf(gx, 0.0f, beta);
    float gi = angle(nin, normalize(n));
    float h = ko_sinf(gi);
    float dh = fabsf(-2.0f / sqrtf(1.0f - h * h));
    float cgi = ko_cosf(gi);
    float sgi = ko_sinf(gi);
    float x1 = sqrtf(ior * ior - sgi * sgi);
    float b1 = x1 / cgi;
    float b2 = ior * ior * cgi / x1;
    float F = fresnel_dielectric(gi, b1, b2);
    float nr = 0.5f * F * dh;
    float ctd = ko_cosf(td);
    float sc = *pdf * nr / (ctd * ctd);
    *out = o1;
    return V(sc, sc, sc);
}

/* d'Eon R lobe (Bsdf.cpp:784-808, 969-1017) */
static v3 deon_r(const shade_ctx_t* s, v3 in, v3 n, float sample[2], const float hu[2], v3* out, float* pdf,
                 int* flags) {
    const obj_t* o = s->obj;
    v3 U = o->u, Vv = o->v, W = o->w;
    float ior = s->m->ior;
    v3 nin = normalize(in);
    v3 in_cyl = world_to_local(in, Vv, U, W);
    float alpha = (-1.0f * (5.0f + 5.0f * hu[0])) * K_DEG2RAD;
    float beta = (5.0f + 5.0f * hu[1]) * K_DEG2RAD;
    (void)sample;
    if ((*flags & F_CYL_T) || (*flags & F_CYL_TR)) { *out = V(0.0f, 0.0f, 1.0f); return V(0.0f, 0.0f, 0.0f); }
    v3 o1 = reflect(vneg(nin), faceforward(n, vneg(nin), n));
    o1 = rotate_rowvec(o1, alpha, Vv);
    *flags = F_SPECULAR;
    v3 oc = world_to_local(o1, Vv, U, W);
    float ti = ko_atan2f(k_hypotf(in_cyl.x, in_cyl.z), in_cyl.y);
    float tr = ko_atan2f(k_hypotf(oc.x, oc.z), oc.y);
    float v = beta * beta;
    float csch = 1.0f / ko_sinhf((1.0f / v) * K_DEG2RAD);
    float dv = v * K_RAD2DEG;
    float e = ko_expf((ko_sinf(-ti) * ko_sinf(tr)) / dv);
    float bes = (float)ko_j0((double)((ko_cosf(-ti) * ko_cosf(tr)) / dv));
    *pdf = (csch / (2.0f * v)) * e * bes;
    float pi_ = ko_atan2f(in_cyl.x, in_cyl.y);
    float pr = ko_atan2f(oc.x, oc.y);
    float dr = 0.25f * fabsf(ko_cosf(pr - pi_ / 2.0f));
    float F = fresnel_dielectric(0.5f * ko_acosf(dot(nin, normalize(o1))), 1.0f, ior);
    float nr = 0.5f * F * dr;
    *out = o1;
    float r = *pdf * nr;
    return V(r, r, r);
}

/* BSDF::sample (Bsdf.cpp:179-184) + localSample dispatch.  Returns reflectance;
 * *valid = 0 when the early `dot(ray_in, normal) == 0` exit fires. */
static v3 bsdf_sample(const shade_ctx_t* s, v3 in, v3 n, float sample[2], const float hu[2], v3* out, float* pdf,
                      int* flags, int* valid) {
    v3 zero = V(0.0f, 0.0f, 0.0f);
    *valid = 1;
    if (dot(in, n) == 0.0f) { *valid = 0; *out = V(0.0f, 0.0f, 1.0f); return zero; }
    const khp_material* m = s->m;
    switch (m->bsdf) {
    case KHP_BSDF_LAMBERTIAN_REFLECTION: {   /* Bsdf.cpp:186-195 */
        int entering = dot(in, n) > 0.0f;
        v3 h = cosine_hemi(sample[0], sample[1]);
        *out = local_to_world_normal(entering ? h : vneg(h), n);
        *pdf = fabsf(dot(*out, n)) * K_ONE_OVER_PI;
        *flags = 0;
        if (*pdf == 0.0f) return zero;
        return vscale(ld3(m->diffuse), K_ONE_OVER_PI);
    }
    case KHP_BSDF_SPECULAR_REFLECTION: {     /* Bsdf.cpp:210-217 */
        *out = reflect(vneg(in), faceforward(n, vneg(in), n));
        *pdf = 1.0f;
        *flags |= F_SPECULAR;
        return vdivs(ld3(m->specular), fabsf(dot(*out, n)));
    }
    case KHP_BSDF_GLOSSY: {                  /* Bsdf.cpp:227-245 */
        float rad = (180.0f - (1.0f - m->roughness) * 180.0f) * K_DEG2RAD;
        v3 ffn = faceforward(n, vneg(in), n);
        v3 refl = reflect(vneg(in), ffn);
        v3 sp = sample_angle(sample[0], sample[1], rad);
        *out = local_to_world_normal(sp, refl);
        if (dot(*out, faceforward(n, vneg(in), n)) < 0.0f) *out = local_to_world_normal(vmul(sp, V(-1.0f, -1.0f, 1.0f)), refl);
        *pdf = 1.0f;
        *flags |= F_SPECULAR;
        return vdivs(ld3(m->specular), fabsf(dot(*out, n)));
    }
    case KHP_BSDF_SPECULAR_TRANSMISSION: {   /* Bsdf.cpp:258-288 */
        int entering = dot(in, n) > 0.0f;
        float ei = entering ? 1.0f : m->ior, et = entering ? m->ior : 1.0f;
        float F = fresnel_dielectric(fabsf(dot(in, n)), ei, et);
        *flags |= F_SPECULAR;
        *out = refract(normalize(vneg(in)), faceforward(n, vneg(in), n), ei / et);
        *pdf = 1.0f;
        if (!is_zero(*out) && !(out->x != out->x)) {
            *flags |= F_TRANSPARENT;
            v3 ft = vscale(ld3(m->volume), 1.0f - F);
            ft = vscale(ft, (ei * ei) / (et * et));
            return vdivs(ft, fabsf(dot(*out, n)));
        }
        return zero;
    }
    case KHP_BSDF_LAMBERTIAN_TRANSMISSION: { /* Bsdf.cpp:298-308 */
        int entering = dot(in, n) > 0.0f;
        v3 h = cosine_hemi(sample[0], sample[1]);
        *out = local_to_world_normal(entering ? vneg(h) : h, n);
        *pdf = fabsf(dot(*out, n)) * K_ONE_OVER_PI;
        *flags = F_TRANSPARENT;
        if (*pdf == 0.0f) return zero;
        return vscale(ld3(m->volume), K_ONE_OVER_PI);
    }
    case KHP_BSDF_GLASS: {                   /* Bsdf.cpp:326-357 */
        int entering = dot(in, n) > 0.0f;
        float ei = entering ? 1.0f : m->ior, et = entering ? m->ior : 1.0f;
        float F = fresnel_dielectric(fabsf(dot(normalize(in), n)), ei, et);
        *flags |= F_SPECULAR;
        v3 nin = normalize(in);
        *out = refract(normalize(vneg(in)), faceforward(n, vneg(nin), n), ei / et);
        if (!is_zero(*out) && sample[1] > F && !(out->x != out->x)) {
            *flags |= F_TRANSPARENT;
            *pdf = 1.0f - F;
            v3 ft = vscale(ld3(m->volume), 1.0f - F);
            ft = vscale(ft, (ei * ei) / (et * et));
            return vdivs(ft, fabsf(dot(*out, n)));
        }
        *out = reflect(normalize(vneg(in)), faceforward(n, vneg(nin), n));
        *pdf = F;
        return vdivs(vscale(ld3(m->specular), F), fabsf(dot(*out, n)));
    }
    case KHP_BSDF_MILK_GLASS: {              /* Bsdf.cpp:367-416 */
        int entering = dot(in, n) > 0.0f;
        float ei = entering ? 1.0f : m->ior, et = entering ? m->ior : 1.0f;
        v3 nin = normalize(in);
        float F = fresnel_dielectric(fabsf(dot(nin, n)), ei, et);
        *flags |= F_SPECULAR;
        v3 refr = refract(normalize(vneg(in)), faceforward(n, vneg(nin), n), ei / et);
        if (!is_zero(refr) && sample[1] > F && !(refr.x != refr.x)) {
            float rad = (180.0f - (1.0f - m->roughness) * 180.0f) * K_DEG2RAD;
            v3 sp = sample_angle(sample[0], sample[1], rad);
            *out = local_to_world_normal(sp, refr);
            if (dot(*out, faceforward(n, vneg(in), n)) > 0.0f) *out = local_to_world_normal(vmul(sp, V(-1.0f, -1.0f, 1.0f)), refr);
            *flags |= F_TRANSPARENT;
            *pdf = 1.0f - F;
            v3 ft = vscale(ld3(m->volume), 1.0f - F);
            ft = vscale(ft, (ei * ei) / (et * et));
            return vdivs(ft, fabsf(dot(*out, n)));
        }
        float rad = (180.0f - (1.0f - m->roughness) * 180.0f) * K_DEG2RAD;
        v3 refl = reflect(vneg(in), faceforward(n, vneg(in), n));
        v3 sp = sample_angle(sample[0], sample[1], rad);
        *out = local_to_world_normal(sp, refl);
        if (dot(*out, faceforward(n, vneg(in), n)) < 0.0f) *out = local_to_world_normal(vmul(sp, V(-1.0f, -1.0f, 1.0f)), refl);
        *pdf = F;
        return vdivs(vscale(ld3(m->specular), F), fabsf(dot(*out, n)));
    }
    case KHP_BSDF_EMISSION:                  /* Bsdf.cpp:427-435 */
        *pdf = 1.0f; *out = zero; *flags = F_EMISSIVE;
        return V(1.0f, 1.0f, 1.0f);
    case KHP_BSDF_TRANSPARENT:               /* Bsdf.cpp:445-454 */
        *out = vneg(in);
        *flags = F_TRANSPARENT | F_SPECULAR;
        *pdf = 1.0f;
        return vdivs(ld3(m->volume), fabsf(dot(*out, n)));
    case KHP_BSDF_MARSCHNER_HAIR:
        return marschner_r(s, in, n, sample, hu, out, pdf, flags);
    case KHP_BSDF_DEON_HAIR:
        return deon_r(s, in, n, sample, hu, out, pdf, flags);
    default:
        *out = V(0.0f, 0.0f, 1.0f); *pdf = 0.0f;
        return zero;
    }
}

/* ======================================================================= */
/*  textures (ABI 6)                                                        */
/* ======================================================================= */
typedef struct { float r, g, b, a; } rgba_t;

/* Texture::getColor (Texture.cpp:243-287).  The wrap `glm::pow(x - floor(x),
 * m_texture_wrap_mode)` is std::pow on doubles (glm `using std::pow`; the mode
 * is an unsigned char).  Out-of-image texel indices (infinite coordinates,
 * undefined in KIRK) are clamped. */
static rgba_t tex_get(const tex_t* t, float x, float y) {
    rgba_t red = {1.0f, 0.0f, 0.0f, 1.0f};
    if (isnan(x) || isnan(y)) return red;
    float ux = x, uy = y;
    if (ux > 1.0 || ux < 0.0) ux = (float)pow((double)(x - floorf(x)), (double)t->wrap);
    if (uy > 1.0 || uy < 0.0) uy = (float)pow((double)(y - floorf(y)), (double)t->wrap);
    int sx = (int)(ux * (int)(t->w - 1));
    int sy = (int)(uy * (int)(t->h - 1));
    if (sx < 0) sx = 0;
    if (sx >= (int)t->w) sx = (int)t->w - 1;
    if (sy < 0) sy = 0;
    if (sy >= (int)t->h) sy = (int)t->h - 1;
    const uint8_t* px = t->data + (size_t)t->ch * ((size_t)sy * t->w + (size_t)sx);
    rgba_t c;
    switch (t->ch) {
    case 4: c.r = px[0] / 255.f; c.g = px[1] / 255.f; c.b = px[2] / 255.f; c.a = px[3] / 255.f; break;
    case 3: c.r = px[0] / 255.f; c.g = px[1] / 255.f; c.b = px[2] / 255.f; c.a = 1.f; break;
    case 2: c.r = c.g = c.b = px[0] / 255.f; c.a = px[1] / 255.f; break;
    default: c.r = c.g = c.b = c.a = px[0] / 255.f; break;
    }
    return c;
}

/* calcTcoord: Cylinder.cpp:239-260, Triangle.cpp:250-254 (bary (1-u-v, u, v)). */
static void obj_tcoord(const obj_t* o, const hit_t* h, v3 loc, float* tu, float* tv) {
    if (o->is_cone) {
        v3 Q = vsub(loc, o->base);
        float u = dot(Q, o->u), v = dot(Q, o->v), w = dot(Q, o->w);
        float r = o->r0 - o->slope * v;
        float tmp = w / r;
        if (tmp < -1.f) tmp = -1.f;
        else if (tmp > 1.f) tmp = 1.f;
        float phi = (u < 0) ? 2.0f * K_PIF - ko_acosf(tmp) : ko_acosf(tmp);
        *tu = phi / 2.f / K_PIF;
        *tv = v / o->height;
    } else {
        float bx = (1.0f - h->bu) - h->bv;
        *tu = (bx * o->tc[0] + h->bu * o->tc[2]) + h->bv * o->tc[4];
        *tv = (bx * o->tc[1] + h->bu * o->tc[3]) + h->bv * o->tc[5];
    }
}

/* Material::getFromParam (Material.cpp:15-23): texel rgb for colours, glm::length
 * of the rgba texel ((r r + g g) + (b b + a a)) for roughness. */
static void material_at(const struct ko_ctx* c, uint32_t mi, float tu, float tv, khp_material* out) {
    *out = c->mats[mi];
    const khp_material_textures* mt = &c->mtex[mi];
    int32_t ids[4] = {mt->diffuse, mt->specular, mt->volume, mt->emission};
    float* dst[4] = {out->diffuse, out->specular, out->volume, out->emission};
    for (int k = 0; k < 4; ++k) {
        if (ids[k] < 0) continue;
        rgba_t t = tex_get(&c->tex[ids[k]], tu, tv);
        dst[k][0] = t.r; dst[k][1] = t.g; dst[k][2] = t.b;
    }
    if (mt->roughness >= 0) {
        rgba_t t = tex_get(&c->tex[mt->roughness], tu, tv);
        out->roughness = sqrtf((t.r * t.r + t.g * t.g) + (t.b * t.b + t.a * t.a));
    }
}

static float glm_sign(float x) { return (float)((0.0f < x) - (x < 0.0f)); }

/* Environment::getColor (Environment.cpp:91-133). */
static v3 env_get(const struct ko_ctx* c, v3 ray_direction) {
    if (c->env_map.type == KHP_ENV_COLOR) return ld3(c->env.color);
    v3 direction = normalize(ray_direction);
    rgba_t t;
    if (c->env_map.type == KHP_ENV_CUBE_MAP) {
        v3 signs = V(glm_sign(direction.x), glm_sign(direction.y), glm_sign(direction.z));
        v3 absolutes = V(fabsf(direction.x), fabsf(direction.y), fabsf(direction.z));
        float max = gmax(gmax(absolutes.x, absolutes.y), absolutes.z);
        int side;
        float uvx, uvy;
        if (max == absolutes.x) {
            side = (int)(0 + 1.5f - 1.5f * signs.x);
            uvx = (direction.z / direction.x + 1) / 2;
            uvy = (direction.y / absolutes.x + 1) / 2;
        } else if (max == absolutes.y) {
            side = (int)(1 + 1.5f - 1.5f * signs.y);
            uvx = (direction.x / absolutes.y + 1) / 2;
            uvy = (direction.z / direction.y + 1) / 2;
        } else {
            side = (int)(2 + 1.5f + 1.5f * signs.z);
            uvx = -(direction.x / direction.z + 1) / 2;
            uvy = (direction.y / absolutes.z + 1) / 2;
        }
        t = tex_get(&c->tex[c->env_map.tex[side]], uvx, uvy);
    } else {
        float m = (float)(2.0 * sqrt(direction.x * direction.x + direction.y * direction.y +
                                     (direction.z + 1.0) * (direction.z + 1.0)));
        float uvx = (float)(direction.x / m + 0.5), uvy = (float)(direction.y / m + 0.5);
        t = tex_get(&c->tex[c->env_map.tex[0]], uvx, uvy);
    }
    return V(t.r, t.g, t.b);
}

/* ======================================================================= */
/*  shaders + integrator                                                    */
/* ======================================================================= */
typedef struct {
    v3 T, color;
    int flags;
    ray_t ray;
} path_t;

/* SimpleShader::calcDirectLight (SimpleShader.h:101-152) == MarschnerHairShader::calcDirectLight
 * (MarschnerHairShader.h:87-138). */
static v3 direct_light(const struct ko_ctx* c, const shade_ctx_t* s, v3 loc, const ray_t* ray, uint32_t key, uint32_t b) {
    v3 zero = V(0.0f, 0.0f, 0.0f);
    if (c->n_lights == 0) return zero;
    int li = (int)((double)draw_u01(key, DIM(b, P_LIGHT_SEL)) * (double)c->n_lights);
    const light_t* L = &c->lights[li];
    float att;
    ray_t h2l = light_dir(L, loc, draw_u01(key, DIM(b, P_LIGHT_0)), draw_u01(key, DIM(b, P_LIGHT_1)), &att);
    v3 lightpos = vadd(h2l.o, h2l.d);
    h2l.o = vadd(h2l.o, vscale(faceforward(s->n, vsub(h2l.o, lightpos), s->n), 1e-4f));
    h2l.d = normalize(h2l.d);
    v3 lc = L->color;
    if (L->color.x > 0.0f || L->color.y > 0.0f || L->color.z > 0.0f) {
        v3 f = bsdf_eval(s, h2l.d, vneg(ray->d));
        float ad = fabsf(dot(h2l.d, s->n));
        lc = V(lc.x * ((att * f.x) * ad), lc.y * ((att * f.y) * ad), lc.z * ((att * f.z) * ad));
        float t_max = length(vsub(lightpos, h2l.o));
        int occ = bvh_any(c, &h2l, t_max, NULL);
        if (!occ) {
            for (uint32_t i = 0; i < c->n_lights; ++i) {
                float t;
                if (light_isect(&c->lights[i], &h2l, &t) && (t < t_max)) { occ = 1; break; }
            }
        }
        lc = vscale(lc, occ ? 0.0f : 1.0f);
        return vadd(zero, lc);
    }
    return zero;
}

static int max3_lt(v3 T, float th) { return gmax(T.x, gmax(T.y, T.z)) < th; }

/* ======================================================================= */
/*  light-path (bidirectional) variant: KIRK's GLSL lbb_construction.compute */
/*  :195-403 and pt_shade.compute:146-201    */
/* ======================================================================= */
#define GL_PI 3.14159265359f          /* inc_random.compute:11, a GLSL float */
#define GL_ONE_OVER_PI 0.31830988618f /* inc_random.compute:12 */
#define GL_DEG2RAD 0.01745329251994329577f
struct lvert {
    int valid;
    v3 pos;   /* vertex position (the light sample point for vertex 0) */
    v3 din;   /* direction of the ray that reached it (0 for vertex 0, lbb_construction.compute:235) */
    v3 hc;    /* hit_color */
};
typedef struct lvert lvert_t;
/* light-path RNG: the path key of subpath (s, light) at sample index k */
static uint32_t lpath_key(uint32_t seed, uint32_t sub, uint32_t k) { return path_key(seed ^ 0x4C504154u, sub, k); }

static v3 gl_cos_hemi(float u, float v) {   /* cosineHemisphereSample, inc_random.compute:50-65 */
    float r = sqrtf(u), th = 2.0f * GL_PI * v;
    float x = r * ko_cosf(th), y = r * ko_sinf(th);
    return V(x, y, sqrtf(gmax(0.0f, (1.0f - x * x) - y * y)));
}
static v3 gl_uniform_sphere(float u, float v) {   /* uniformSphereSample, inc_random.compute:75-81 */
    float phi = v * 2.0f * GL_PI, ct = 2.0f * u - 1.0f;
    float st = sqrtf(gmax(0.0f, 1.0f - ct * ct));
    return V(st * ko_cosf(phi), st * ko_sinf(phi), ct);
}
static v3 gl_sample_angle(float u, float v, float max_angle) {   /* sampleAngle, inc_random.compute:67-73 */
    float phi = v * 2.0f * GL_PI, ct = 1.0f - u * (1.0f - ko_cosf(max_angle));
    float st = sqrtf(1.0f - ct * ct);
    return V(ko_cosf(phi) * st, ko_sinf(phi) * st, ct);
}
/* the (s, t, n) frame of lbb_construction.compute:42-45, and localToWorld (BSDF/header.compute:23-26) */
static v3 gl_to_world(v3 v, v3 n) {
    v3 s = normalize(n.y * n.y > n.x * n.x ? V(0.0f, n.z, -n.y) : V(-n.z, 0.0f, n.x));
    v3 t = normalize(cross(n, s));
    return vadd(vadd(vscale(s, v.x), vscale(t, v.y)), vscale(n, v.z));
}
/* calcLightBounce{Point,Sun,Spot,Quad} (lbb_construction.compute:35-141): the ray leaving the light */
static ray_t gl_light_ray(const light_t* L, float a0, float a1, float b0, float b1) {
    ray_t r;
    if (L->kind == KHP_LIGHT_POINT) {
        v3 n = gl_uniform_sphere(a0, a1);
        r.o = vadd(L->position, vscale(n, L->radius));
        r.d = gl_to_world(gl_cos_hemi(b0, b1), n);
    } else if (L->kind == KHP_LIGHT_SUN) {
        v3 pos = vadd(vneg(L->direction), vscale(gl_uniform_sphere(a0, a1), L->radius));
        v3 dn = normalize(pos);
        r.o = vadd(pos, vscale(dn, 1e16f));
        r.d = L->direction;
    } else if (L->kind == KHP_LIGHT_SPOT) {
        v3 pr = gl_cos_hemi(a0, a1);
        pr.z = 0.0f;
        pr = vscale(pr, L->radius);
        v3 dr = gl_sample_angle(b0, b1, L->outer * GL_DEG2RAD);
        r.o = vadd(L->position, gl_to_world(pr, L->direction));
        r.d = gl_to_world(dr, L->direction);
    } else {
        v3 x1 = vadd(L->vert[0], vscale(vsub(L->vert[1], L->vert[0]), a0));
        v3 x2 = vadd(L->vert[3], vscale(vsub(L->vert[2], L->vert[3]), a0));
        r.o = vadd(x1, vscale(vsub(x2, x1), a1));
        r.d = gl_to_world(gl_cos_hemi(b0, b1), L->direction);
    }
    r.d = normalize(r.d);
    return r;
}
/* the light's attenuation_linear / _quadratic as the GLSL light bounce carries them (0 for spot and sun) */
static void gl_light_att(const light_t* L, float* al, float* aq) {
    int carries = L->kind == KHP_LIGHT_POINT || L->kind == KHP_LIGHT_QUAD;
    *al = carries ? L->l : 0.0f;
    *aq = carries ? L->q : 0.0f;
}
/* angularAttenuation (inc_light.compute:207-237) */
static float gl_ang_att(const light_t* L, v3 d) {
    if (L->kind == KHP_LIGHT_SPOT) {
        float ang = ko_acosf(dot(normalize(vneg(d)), L->direction)) * K_RAD2DEG;
        return 1.0f - gclamp((ang - L->inner) / (L->outer - L->inner), 0.0f, 1.0f);
    }
    if (L->kind == KHP_LIGHT_QUAD) return dot(normalize(vneg(d)), L->direction);
    return 1.0f;
}

/* One light subpath (generatePrimaryLightRays + traceLightRays + shadeLightRays,
 * lbb_construction.compute:195-403): J vertices, the first on the light. */
static void light_subpath(const struct ko_ctx* c, uint32_t seed, uint32_t k, uint32_t s, uint32_t li, lvert_t* out) {
    const khp_bdpt_params* bd = &c->bd;
    const uint32_t J = bd->vertices, L = c->n_lights;
    const light_t* Lt = &c->lights[li];
    const uint32_t key = lpath_key(seed, s * L + li, k);
    memset(out, 0, sizeof(lvert_t) * J);   /* invalid vertices are all-zero records */
    ray_t r = gl_light_ray(Lt, draw_u01(key, DIM(0, P_LIGHT_0)), draw_u01(key, DIM(0, P_LIGHT_1)),
                           draw_u01(key, DIM(0, P_BSDF_0)), draw_u01(key, DIM(0, P_BSDF_1)));
    out[0].valid = 1;
    out[0].pos = r.o;
    out[0].din = V(0.0f, 0.0f, 0.0f);
    out[0].hc = V(GL_ONE_OVER_PI, GL_ONE_OVER_PI, GL_ONE_OVER_PI);
    float al, aq, dist = 0.0f;
    gl_light_att(Lt, &al, &aq);
    for (uint32_t j = 1; j < J; ++j) {
        hit_t h;
        if (!bvh_closest(c, &r, &h, NULL)) return;   /* traceLightRays: no hit ends the subpath */
        const obj_t* o = &c->obj[h.obj];
        v3 n = obj_normal(o, &r, &h), pos = follow(&r, h.lambda);
        const khp_material* m = &c->mats[o->mat];
        khp_material mtx;
        if (c->textured) {
            float tu, tv;
            obj_tcoord(o, &h, pos, &tu, &tv);
            material_at(c, o->mat, tu, tv, &mtx);
            m = &mtx;
        }
        shade_ctx_t sc; sc.obj = o; sc.m = m; sc.n = n;
        dist = dist + length(vsub(pos, r.o));
        float att = 1.0f / ((1.0f + dist * al) + (dist * dist) * aq);
        v3 in = vneg(r.d), out_d = V(0.0f, 0.0f, 0.0f), f = V(0.0f, 0.0f, 0.0f);
        float pdf = 0.0f;
        int fl = 0;
        if (!(dot(in, n) == 0.0f)) {   /* reflectance (BSDF/header.compute:48-56) */
            float smp[2] = {draw_u01(key, DIM(j, P_BSDF_0)), draw_u01(key, DIM(j, P_BSDF_1))};
            float hu[2] = {draw_u01(key, DIM(j, P_HAIR_ALPHA)), draw_u01(key, DIM(j, P_HAIR_BETA))};
            int valid;
            f = bsdf_sample(&sc, in, n, smp, hu, &out_d, &pdf, &fl, &valid);
        }
        v3 hc = vmul(out[j - 1].hc, f);
        v3 w = vsub(pos, out[j - 1].pos);   /* convertDensity (:280-299), previous vertex = its position */
        float ww = dot(w, w);
        if (ww == 0.0f) pdf = 0.0f;
        else pdf = pdf * fabsf(dot(n, vscale(w, sqrtf(1.0f / ww))));
        hc = vscale(hc, gclamp(fabsf(dot(out_d, n)) * pdf, 0.0f, 1.0f));
        if ((fl & F_EMISSIVE) == F_EMISSIVE) return;
        if (is_zero(hc) || pdf <= bd->min_pdf || att <= 0.0001f) return;
        out[j].valid = 1;
        out[j].pos = pos;
        out[j].din = r.d;
        out[j].hc = hc;
        r = make_ray(vadd(pos, vscale(out_d, bd->bounce_bias)), out_d);
    }
}

/* The subpaths of sample indices [k0, k0+nk) (before the render's worker threads start). */
static int build_light_paths(struct ko_ctx* c, uint32_t seed, uint32_t k0, uint32_t nk) {
    const uint32_t Ns = c->bd.light_paths, L = c->n_lights, J = c->bd.vertices;
    size_t n = (size_t)nk * Ns * L * J;
    if (n > c->lv_cap) {
        free(c->lv);
        c->lv = (lvert_t*)malloc(sizeof(lvert_t) * (n ? n : 1));
        if (!c->lv) { c->lv_cap = 0; return KHP_ENOMEM; }
        c->lv_cap = n;
    }
    for (uint32_t q = 0; q < nk; ++q)
        for (uint32_t s = 0; s < Ns; ++s)
            for (uint32_t li = 0; li < L; ++li)
                light_subpath(c, seed, k0 + q, s, li, c->lv + (((size_t)q * Ns + s) * L + li) * J);
    c->lv_k0 = k0;
    c->lv_nk = nk;
    return KHP_OK;
}

/* shadeBDPTImagePlane (pt_shade.compute:17-97): connect every valid vertex of one
 * subpath (chosen with the sample's own draws at dims IMG_DIM) to the sample's
 * point on the sensor; the unoccluded importance-weighted terms, summed in
 * vertex order, are the path's first colour add. */
#define IMG_BOUNCE 4095u
static v3 bdpt_image_plane(const struct ko_ctx* c, uint32_t W, uint32_t H, v3 sensor, uint32_t key, uint32_t k) {
    v3 dl = V(0.0f, 0.0f, 0.0f);
    const khp_bdpt_params* bd = &c->bd;
    const uint32_t Ns = bd->light_paths, L = c->n_lights, J = bd->vertices;
    uint32_t sp = (uint32_t)((float)Ns * draw_u01(key, DIM(IMG_BOUNCE, P_LIGHT_0)));
    uint32_t li = (uint32_t)((float)L * draw_u01(key, DIM(IMG_BOUNCE, P_LIGHT_SEL)));
    if (sp >= Ns) sp = Ns - 1;
    if (li >= L) li = L - 1;
    const khp_camera* cam = &c->cam;
    v3 axs = vscale(ld3(cam->axis_x), cam->pixel_size), ays = vscale(ld3(cam->axis_y), cam->pixel_size);
    float a = length(cross(vscale(ays, (float)H), vscale(axs, (float)W)));   /* sensor area */
    v3 cn = normalize(cross(ays, axs));                                        /* camera normal */
    const lvert_t* v = c->lv + (((size_t)(k - c->lv_k0) * Ns + sp) * L + li) * J;
    for (uint32_t j = 0; j < J; ++j) {
        if (!v[j].valid) continue;
        v3 lp;
        if (bd->image_plane == 1) {
            /* as written (pt_shade.compute:38-44): pos = light_bounce.ray.origin, target
             * pos + debug.bias * light_bounce.ray.direction.  Record j's ray
             * (lbb_construction.compute:229-235, 391-395): j = 0 (light point, 0),
             * j = 1 (light point, d0), j >= 2 (pos_{j-1} + bounce_bias * out_{j-1},
             * out_{j-1}); din_j holds that direction (0 for j = 0). */
            v3 org = j >= 2 ? vadd(v[j - 1].pos, vscale(v[j].din, bd->bounce_bias)) : v[j >= 1 ? j - 1 : 0].pos;
            lp = vadd(org, vscale(v[j].din, bd->bias));
        } else {   /* 2: the vertex itself, pulled back like the hit connections' target */
            lp = vsub(v[j].pos, vscale(v[j].din, bd->bounce_bias));
        }
        v3 d = vsub(lp, sensor);
        float t = length(d);
        ray_t vis;
        vis.o = sensor;
        vis.d = normalize(d);
        float ct = dot(cn, vis.d);
        float we = 1.0f / ((((a * ct) * ct) * ct) * ct);
        float npdf = (t * t) / fabsf(dot(cn, vis.d));
        if (ct <= 0.0f) we = 0.0f;
        v3 cj = vdivs(vdivs(vscale(v[j].hc, we), npdf), (float)(j + 1));
        int occ = bvh_any(c, &vis, t, NULL);
        if (!occ) {
            for (uint32_t i = 0; i < c->n_lights; ++i) {
                float tl;
                if (light_isect(&c->lights[i], &vis, &tl) && (tl < t)) { occ = 1; break; }
            }
        }
        if (!occ) dl = vadd(dl, cj);
    }
    /* added like a connection group's term: (0 + dl * 1) + 0 */
    return vadd(vadd(V(0.0f, 0.0f, 0.0f), vmul(dl, V(1.0f, 1.0f, 1.0f))), V(0.0f, 0.0f, 0.0f));
}

/* pt_shade.compute:146-201: connect the hit to every valid vertex of one subpath
 * (subpath and light chosen with the path's light-select draws).  Returns the
 * sum of the unoccluded contributions hit_color * light colour * |cos| * f / (j + 1 + b). */
static v3 bdpt_connect(const struct ko_ctx* c, const shade_ctx_t* s, v3 loc, const ray_t* ray, uint32_t key, uint32_t b,
                       uint32_t k) {
    v3 dl = V(0.0f, 0.0f, 0.0f);
    const khp_bdpt_params* bd = &c->bd;
    const uint32_t Ns = bd->light_paths, L = c->n_lights, J = bd->vertices;
    if (L == 0) return dl;
    uint32_t sp = (uint32_t)((float)Ns * draw_u01(key, DIM(b, P_LIGHT_0)));
    uint32_t li = (uint32_t)((float)L * draw_u01(key, DIM(b, P_LIGHT_SEL)));
    if (sp >= Ns) sp = Ns - 1;
    if (li >= L) li = L - 1;
    const light_t* Lt = &c->lights[li];
    const lvert_t* v = c->lv + (((size_t)(k - c->lv_k0) * Ns + sp) * L + li) * J;
    for (uint32_t j = 0; j < J; ++j) {
        if (!v[j].valid) continue;
        v3 lp = vsub(v[j].pos, vscale(v[j].din, bd->bounce_bias));
        v3 lc = j == 0 ? vscale(Lt->color, gl_ang_att(Lt, vsub(lp, loc))) : Lt->color;
        ray_t sh;
        sh.o = vadd(loc, vscale(s->n, bd->bias));
        sh.d = normalize(vsub(lp, loc));
        float t_max = length(vsub(lp, sh.o));
        lc = vscale(lc, fabsf(dot(sh.d, s->n)));
        lc = vmul(lc, bsdf_eval(s, vneg(ray->d), sh.d));
        v3 cj = vdivs(vmul(v[j].hc, lc), (float)(j + 1 + b));
        int occ = bvh_any(c, &sh, t_max, NULL);
        if (!occ) {   /* intersectsAnyWithLights (inc_light.compute:508-535); the sun is never hit */
            for (uint32_t i = 0; i < c->n_lights; ++i) {
                float t;
                if (light_isect(&c->lights[i], &sh, &t) && (t < t_max)) { occ = 1; break; }
            }
        }
        if (!occ) dl = vadd(dl, cj);
    }
    return dl;
}

/* One sample of one pixel: generatePrimaryRays + traceRays + traceRay + shaders
 * (CPU_PathTracer.cpp:118-209; SimpleShader.h:31-98; MarschnerHairShader.h:31-84;
 *  LightShader.h:20-25; EnvironmentShader.h:20-26). */
static v3 trace_sample(const struct ko_ctx* c, const khp_render_params* p, uint32_t x, uint32_t y, uint32_t sample) {
    uint32_t pixel = y * p->width + x;
    uint32_t key = path_key(p->seed, pixel, sample);
    const khp_camera* cam = &c->cam;
    float u1 = draw_u01(key, DIM(0, P_CAM_X)), u2 = draw_u01(key, DIM(0, P_CAM_Y));
    float s1 = ((float)x + u1) * cam->pixel_size, s2 = ((float)y + u2) * cam->pixel_size;
    v3 dir = vsub(vadd(vadd(ld3(cam->bottom_left), vscale(ld3(cam->axis_x), s1)), vscale(ld3(cam->axis_y), s2)),
                  ld3(cam->position));
    path_t P;
    P.ray = make_ray(ld3(cam->position), dir);
    P.T = V(1.0f, 1.0f, 1.0f);
    P.color = V(0.0f, 0.0f, 0.0f);
    P.flags = 0;
    if (c->bd.enabled && c->bd.image_plane && c->n_lights > 0) {
        v3 sensor = vadd(vadd(ld3(cam->bottom_left), vscale(ld3(cam->axis_x), s1)), vscale(ld3(cam->axis_y), s2));
        P.color = vadd(P.color, bdpt_image_plane(c, p->width, p->height, sensor, key, sample));
    }
    for (uint32_t b = 0; b < p->depth; ++b) {
        if (is_zero(P.T)) break;
        if (is_zero(P.ray.d)) break;   /* traceRay lambda=-1 guard (CPU_PathTracer.cpp:172-174); unreachable */
        hit_t h;
        int is_hit = bvh_closest(c, &P.ray, &h, NULL);
        v3 n = V(0.0f, 0.0f, 0.0f);
        if (is_hit) n = obj_normal(&c->obj[h.obj], &P.ray, &h);
        float t_lights = FLT_MAX;
        int t_index = -1;
        for (uint32_t li = 0; li < c->n_lights; ++li) {
            float t = FLT_MAX;
            if (light_isect(&c->lights[li], &P.ray, &t)) {
                t_lights = gmin(t_lights, t);
                t_index = (t == t_lights) ? (int)li : t_index;
            }
        }
        int light_hit = 0;
        if (t_lights < h.lambda) { h.lambda = t_lights; light_hit = 1; }
        if (h.lambda == FLT_MAX) {          /* EnvironmentShader::shade */
            P.color = vadd(P.color, vmul(env_get(c, P.ray.d), P.T));
            P.T = V(0.0f, 0.0f, 0.0f);
            continue;
        }
        if (light_hit) {                    /* LightShader::shade */
            v3 Le = light_emit(&c->lights[t_index], P.ray.d);
            P.color = vadd(P.color, vmul(Le, P.T));
            P.T = V(0.0f, 0.0f, 0.0f);
            continue;
        }
        const obj_t* o = &c->obj[h.obj];
        const khp_material* m = &c->mats[o->mat];
        khp_material mtx;
        if (c->textured) {   /* traceRay: calcTcoord (CPU_PathTracer.cpp:178-179), then fetchParameter* */
            float tu, tv;
            obj_tcoord(o, &h, follow(&P.ray, h.lambda), &tu, &tv);
            material_at(c, o->mat, tu, tv, &mtx);
            m = &mtx;
        }
#ifdef KO_DEBUG
        if (getenv("KO_DEBUG") && (int)x == atoi(getenv("KO_DEBUG")) && (int)y == atoi(getenv("KO_DEBUGY")))
            fprintf(stderr, "s%u b%u obj %d cone %d lambda %g T %g %g %g C %g %g %g n %g %g %g d %g %g %g dn %g\n", sample, b, h.obj,
                    o->is_cone, h.lambda, P.T.x, P.T.y, P.T.z, P.color.x, P.color.y, P.color.z, n.x, n.y, n.z,
                    P.ray.d.x, P.ray.d.y, P.ray.d.z, dot(n, P.ray.d));
#endif
        shade_ctx_t s; s.obj = o; s.m = m; s.n = n;
        v3 loc = follow(&P.ray, h.lambda);
        float hu[2] = {draw_u01(key, DIM(b, P_HAIR_ALPHA)), draw_u01(key, DIM(b, P_HAIR_BETA))};
        v3 counter = vneg(normalize(P.ray.d));
        if (m->shader == KHP_SHADER_MARSCHNER_HAIR) {   /* MarschnerHairShader::shade */
            float sample2[2] = {0.0f, 0.0f};
            v3 out; float pdf = 0.0f; int valid;
            v3 refl = bsdf_sample(&s, counter, n, sample2, hu, &out, &pdf, &P.flags, &valid);
            v3 off = vscale(out, 1e-4f);
            if (!(P.flags & F_SPECULAR)) off = faceforward(vneg(vscale(n, 1e-4f)), n, out);
            ray_t ray_in = P.ray;
            P.ray = make_ray(vadd(loc, off), out);
            if ((P.flags & F_CYL_T) || (P.flags & F_CYL_TR)) continue;
            v3 ev = bsdf_eval(&s, n, n);
            v3 amb = vmul(ld3(c->env.ambient), vscale(ev, K_ONE_OVER_PI));
            v3 dl = c->bd.enabled ? bdpt_connect(c, &s, loc, &ray_in, key, b, sample)
                                  : direct_light(c, &s, loc, &ray_in, key, b);
            v3 acc = vadd(vadd(V(0.0f, 0.0f, 0.0f), vmul(dl, P.T)), vmul(amb, P.T));
            if (is_zero(refl) || pdf <= 1E-4f || max3_lt(P.T, 0.01f)) P.T = V(0.0f, 0.0f, 0.0f);
            else {
                float ac = fabsf(ko_cosf(sample2[0]));
                P.T = vmul(P.T, vscale(vscale(refl, 3.0f), ac));
            }
            P.color = vadd(P.color, acc);
        } else {                                          /* SimpleShader::shade */
            float sample2[2] = {draw_u01(key, DIM(b, P_BSDF_0)), draw_u01(key, DIM(b, P_BSDF_1))};
            v3 emitted = ld3(m->emission);
            v3 ev = bsdf_eval(&s, n, n);
            v3 amb = vmul(ld3(c->env.ambient), vscale(ev, K_ONE_OVER_PI));
            v3 dl = c->bd.enabled ? bdpt_connect(c, &s, loc, &P.ray, key, b, sample)
                                  : direct_light(c, &s, loc, &P.ray, key, b);
            v3 acc = vadd(vadd(V(0.0f, 0.0f, 0.0f), vmul(dl, P.T)), vmul(amb, P.T));
            v3 out; float pdf = 0.0f; int fl = 0, valid;
            v3 refl = bsdf_sample(&s, counter, n, sample2, hu, &out, &pdf, &fl, &valid);
            if (is_zero(refl) || pdf <= 1E-4f || max3_lt(P.T, 0.01f)) {
                P.T = V(0.0f, 0.0f, 0.0f);
                P.color = vadd(P.color, acc);
                continue;
            }
            if ((fl & F_EMISSIVE) == F_EMISSIVE) {
                acc = vadd(acc, vmul(emitted, P.T));
                P.T = V(0.0f, 0.0f, 0.0f);
                P.color = vadd(P.color, acc);
                continue;
            }
            float ad = fabsf(dot(out, n));
            P.T = vmul(P.T, vdivs(vscale(refl, ad), pdf));
            P.flags = fl;
            v3 off = vscale(out, 1e-4f);
            if ((fl & F_SPECULAR) != F_SPECULAR) off = faceforward(vneg(vscale(n, 1e-4f)), n, out);
            P.ray = make_ray(vadd(loc, off), out);
            P.color = vadd(P.color, acc);
        }
    }
    return P.color;
}

/* ======================================================================= */
/*  public API                                                              */
/* ======================================================================= */
int ko_create(ko_ctx** out, const khp_scene* s) {
    *out = NULL;
    if (!s) return KHP_EINVAL;
    struct ko_ctx* c = (struct ko_ctx*)calloc(1, sizeof(struct ko_ctx));
    c->n_tris = s->n_tris; c->n_cones = s->n_cones;
    c->n_obj = s->n_tris + s->n_cones;
    if (c->n_obj == 0) { free(c); return KHP_EINVAL; }   /* "Your scene is empty!" (BoundingBox.cpp:121-122) */
    c->obj = (obj_t*)malloc(sizeof(obj_t) * c->n_obj);
    for (uint32_t i = 0; i < s->n_tris; ++i) {
        const float* v = s->tri_v + 9 * (size_t)i;
        const float* n = s->tri_n + 9 * (size_t)i;
        tri_ctor(&c->obj[i], ld3(v), ld3(v + 3), ld3(v + 6), ld3(n), ld3(n + 3), ld3(n + 6),
                 s->tri_uv ? s->tri_uv + 6 * (size_t)i : NULL);
        c->obj[i].mat = s->tri_mat[i];
        /* Object::setU/V/W: the fiber's frame for fiberToTriangles fur (CPU_Scene.cpp:297-319),
         * zero for plain triangles (uninitialised glm::vec3 in KIRK) */
        const float* f = s->tri_frame ? s->tri_frame + 9 * (size_t)i : NULL;
        c->obj[i].u = f ? ld3(f) : V(0.0f, 0.0f, 0.0f);
        c->obj[i].v = f ? ld3(f + 3) : V(0.0f, 0.0f, 0.0f);
        c->obj[i].w = f ? ld3(f + 6) : V(0.0f, 0.0f, 0.0f);
    }
    for (uint32_t i = 0; i < s->n_cones; ++i) {
        const float* b = s->cone_base_r0 + 4 * (size_t)i;
        const float* a = s->cone_apex_r1 + 4 * (size_t)i;
        obj_t* o = &c->obj[s->n_tris + i];
        const float* M = NULL;
        if (s->n_cone_models) {
            uint32_t k = s->cone_model ? s->cone_model[i] : 0u;
            if (k >= s->n_cone_models) { free(c->obj); free(c); return KHP_EINVAL; }
            M = s->cone_models + 16 * (size_t)k;
        }
        cone_ctor(o, ld3(b), ld3(a), b[3], a[3], M);
        o->mat = s->cone_mat[i];
    }
    c->n_mats = s->n_materials;
    c->mats = (khp_material*)malloc(sizeof(khp_material) * (c->n_mats ? c->n_mats : 1));
    memcpy(c->mats, s->materials, sizeof(khp_material) * c->n_mats);
    for (uint32_t i = 0; i < c->n_obj; ++i)
        if (c->obj[i].mat >= c->n_mats) { ko_destroy(c); return KHP_EINVAL; }
    c->n_lights = s->n_lights;
    c->lights = (light_t*)malloc(sizeof(light_t) * (c->n_lights ? c->n_lights : 1));
    for (uint32_t i = 0; i < c->n_lights; ++i) light_init(&c->lights[i], &s->lights[i]);
    c->env = s->env;
    c->cam = s->camera;
    c->env_map = s->env_map;
    c->n_tex = s->n_textures;
    c->tex = (tex_t*)calloc(c->n_tex ? c->n_tex : 1, sizeof(tex_t));
    for (uint32_t i = 0; i < c->n_tex; ++i) {
        const khp_texture* t = &s->textures[i];
        size_t nb = (size_t)t->width * t->height * t->channels;
        c->tex[i].w = t->width; c->tex[i].h = t->height; c->tex[i].ch = t->channels; c->tex[i].wrap = t->wrap_mode;
        c->tex[i].data = (uint8_t*)malloc(nb ? nb : 1);
        memcpy(c->tex[i].data, t->data, nb);
        if (t->channels < 1 || t->channels > 4 || t->width == 0 || t->height == 0) { ko_destroy(c); return KHP_EINVAL; }
    }
    c->mtex = (khp_material_textures*)malloc(sizeof(khp_material_textures) * (c->n_mats ? c->n_mats : 1));
    for (uint32_t i = 0; i < c->n_mats; ++i) {
        khp_material_textures none = {-1, -1, -1, -1, -1};
        c->mtex[i] = s->material_textures ? s->material_textures[i] : none;
        const int32_t* k = &c->mtex[i].diffuse;
        for (int j = 0; j < 5; ++j) {
            if (k[j] >= (int32_t)c->n_tex || k[j] < -1) { ko_destroy(c); return KHP_EINVAL; }
            if (k[j] >= 0) c->textured = 1;
        }
    }
    if (c->env_map.type == KHP_ENV_CUBE_MAP || c->env_map.type == KHP_ENV_SPHERE_MAP) {
        for (int j = 0; j < (c->env_map.type == KHP_ENV_CUBE_MAP ? 6 : 1); ++j)
            if (c->env_map.tex[j] < 0 || c->env_map.tex[j] >= (int32_t)c->n_tex) { ko_destroy(c); return KHP_EINVAL; }
    } else if (c->env_map.type != KHP_ENV_COLOR) {
        ko_destroy(c);
        return KHP_EINVAL;
    }
    /* BVH::addBaseDataStructure (CPU_BVH.cpp:16-44) */
    c->ids = (uint32_t*)malloc(sizeof(uint32_t) * c->n_obj);
    box_t cb = box_empty();
    for (uint32_t i = 0; i < c->n_obj; ++i) { box_grow_pt(&cb, c->obj[i].centroid); c->ids[i] = i; }
    split(c, 0, c->n_obj - 1, &cb, 1);
    *out = c;
    return KHP_OK;
}

void ko_destroy(ko_ctx* c) {
    if (!c) return;
    free(c->obj); free(c->mats); free(c->lights); free(c->nodes); free(c->ids); free(c->lv);
    for (uint32_t i = 0; i < c->n_tex; ++i) free(c->tex[i].data);
    free(c->tex); free(c->mtex);
    free(c);
}

static int owns_pixel(const khp_render_params* p, uint32_t x, uint32_t y) {
    if (p->tile_nranks <= 1) return 1;
    uint32_t T = p->tile_size ? p->tile_size : 64;
    uint32_t tiles_x = (p->width + T - 1) / T;
    uint32_t tid = (y / T) * tiles_x + (x / T);
    return (tid % p->tile_nranks) == p->tile_rank;
}

typedef struct {
    ko_ctx* c;
    const khp_render_params* p;
    float* out;
    uint32_t y0, y1, ystep;
    int tid, nth;
} job_t;

static void* render_worker(void* arg) {
    job_t* j = (job_t*)arg;
    const khp_render_params* p = j->p;
    for (uint32_t y = j->y0 + (uint32_t)j->tid * j->ystep; y < j->y1; y += (uint32_t)j->nth * j->ystep) {
        for (uint32_t x = 0; x < p->width; ++x) {
            if (!owns_pixel(p, x, y)) continue;
            float* o = j->out + 3 * ((size_t)y * p->width + x);
            for (uint32_t s = 0; s < p->spp; ++s) {
                uint32_t k = p->first_sample + s;
                v3 col = trace_sample(j->c, p, x, y, k);
                /* PathTracer::drawTexture running mean (CPU_PathTracer.cpp:68-75) */
                if (k == 0) { o[0] = col.x; o[1] = col.y; o[2] = col.z; }
                else {
                    float kk = (float)(k + 1);
                    o[0] = o[0] + (col.x - o[0]) / kk;
                    o[1] = o[1] + (col.y - o[1]) / kk;
                    o[2] = o[2] + (col.z - o[2]) / kk;
                }
            }
        }
    }
    return NULL;
}

int ko_render_rows(ko_ctx* c, const khp_render_params* p, int n_threads, uint32_t y0, uint32_t y1, float* out_rgb) {
    return ko_render_rows_step(c, p, n_threads, y0, y1, 1, out_rgb);
}

int ko_render_rows_step(ko_ctx* c, const khp_render_params* p, int n_threads, uint32_t y0, uint32_t y1,
                        uint32_t ystep, float* out_rgb) {
    if (!c || !p || !out_rgb || p->width == 0 || p->height == 0 || ystep == 0) return KHP_EINVAL;
    if (y1 > p->height) y1 = p->height;
    if (c->bd.enabled) {
        int e = build_light_paths(c, p->seed, p->first_sample, p->spp);
        if (e != KHP_OK) return e;
    }
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    job_t jobs[256];
    for (int t = 0; t < n_threads; ++t) {
        jobs[t].c = c; jobs[t].p = p; jobs[t].out = out_rgb; jobs[t].y0 = y0; jobs[t].y1 = y1; jobs[t].ystep = ystep;
        jobs[t].tid = t; jobs[t].nth = n_threads;
        if (n_threads > 1) pthread_create(&th[t], NULL, render_worker, &jobs[t]);
    }
    if (n_threads == 1) render_worker(&jobs[0]);
    else for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    return KHP_OK;
}

int ko_render(ko_ctx* c, const khp_render_params* p, int n_threads, float* out_rgb) {
    return ko_render_rows(c, p, n_threads, 0, p ? p->height : 0, out_rgb);
}

int ko_trace_closest(ko_ctx* c, uint32_t n, const float* orig, const float* dir, float* t_out, int32_t* obj_out,
                     float* uv_out, uint64_t* node_visits, uint64_t* prim_tests) {
    trav_stats_t st = {0, 0, NULL, 0, 0, 0};
    for (uint32_t i = 0; i < n; ++i) {
        ray_t r = make_ray(ld3(orig + 3 * (size_t)i), ld3(dir + 3 * (size_t)i));
        hit_t h;
        bvh_closest(c, &r, &h, &st);
        t_out[i] = h.lambda;
        obj_out[i] = h.obj;
        if (uv_out) { uv_out[2 * i] = h.bu; uv_out[2 * i + 1] = h.bv; }
    }
    if (node_visits) *node_visits = st.nodes;
    if (prim_tests) *prim_tests = st.prims;
    return KHP_OK;
}

/* Dev-tool hook (tools/treelet_sim.py): ko_trace_closest that also records, per
 * ray, the preorder ids of the nodes KIRK's traversal visits, in visit order.
 * offsets[n+1]: ray i's visits are log[offsets[i], offsets[i+1]); entries past
 * cap are counted but not stored. */
int ko_trace_closest_log(ko_ctx* c, uint32_t n, const float* orig, const float* dir, float* t_out, int32_t* log,
                         uint64_t cap, uint64_t* offsets) {
    trav_stats_t st = {0, 0, log, 0, cap, 0};
    /* a log entry packs the node id into bits 0..24 and the deferred far-child
     * count into bits 25..31: a larger tree would alias ids and counts */
    if (c->n_nodes >= (1u << 25)) return KHP_EINVAL;
    for (uint32_t i = 0; i < n; ++i) {
        offsets[i] = st.log_n;
        ray_t r = make_ray(ld3(orig + 3 * (size_t)i), ld3(dir + 3 * (size_t)i));
        hit_t h;
        bvh_closest(c, &r, &h, &st);
        t_out[i] = h.lambda;
    }
    offsets[n] = st.log_n;
    return KHP_OK;
}

int ko_trace_any(ko_ctx* c, uint32_t n, const float* orig, const float* dir, const float* tmax, uint8_t* hit_out) {
    for (uint32_t i = 0; i < n; ++i) {
        ray_t r = make_ray(ld3(orig + 3 * (size_t)i), ld3(dir + 3 * (size_t)i));
        hit_out[i] = (uint8_t)bvh_any(c, &r, tmax[i], NULL);
    }
    return KHP_OK;
}

uint32_t ko_n_objects(ko_ctx* c) { return c->n_obj; }

int ko_set_bdpt(ko_ctx* c, const khp_bdpt_params* p) {
    if (!c || !p) return KHP_EINVAL;
    if (p->enabled && (p->light_paths < 1 || p->light_paths > 65536 || p->vertices < 1 || p->vertices > 16))
        return KHP_EINVAL;
    if (p->image_plane > 2) return KHP_EINVAL;
    c->bd = *p;
    return KHP_OK;
}

/* The light subpaths of sample index k (test hook): [light_paths][n_lights][vertices]
 * records of 10 floats: valid, pos.xyz, din.xyz, hit_color.xyz. */
int ko_light_paths(ko_ctx* c, uint32_t seed, uint32_t k, float* out10) {
    if (!c || !c->bd.enabled) return KHP_EINVAL;
    int e = build_light_paths(c, seed, k, 1);
    if (e != KHP_OK) return e;
    size_t n = (size_t)c->bd.light_paths * c->n_lights * c->bd.vertices;
    for (size_t i = 0; i < n; ++i) {
        const lvert_t* v = &c->lv[i];
        float r[10] = {(float)v->valid, v->pos.x, v->pos.y, v->pos.z, v->din.x, v->din.y, v->din.z, v->hc.x, v->hc.y, v->hc.z};
        memcpy(out10 + 10 * i, r, sizeof(r));
    }
    return KHP_OK;
}

void ko_object_bounds(ko_ctx* c, float* o9) {
    for (uint32_t i = 0; i < c->n_obj; ++i) {
        const obj_t* o = &c->obj[i];
        float* d = o9 + 9 * (size_t)i;
        d[0] = o->bmin.x; d[1] = o->bmin.y; d[2] = o->bmin.z;
        d[3] = o->bmax.x; d[4] = o->bmax.y; d[5] = o->bmax.z;
        d[6] = o->centroid.x; d[7] = o->centroid.y; d[8] = o->centroid.z;
    }
}

/* Test hooks (ABI-6 KATs): Environment::getColor and Texture::getColor of the scene's textures. */
void ko_env_color(ko_ctx* c, const float* dir, float* rgb) {
    v3 e = env_get(c, ld3(dir));
    rgb[0] = e.x; rgb[1] = e.y; rgb[2] = e.z;
}

void ko_tex_color(ko_ctx* c, uint32_t t, float x, float y, float* rgba) {
    rgba_t v = tex_get(&c->tex[t], x, y);
    rgba[0] = v.r; rgba[1] = v.g; rgba[2] = v.b; rgba[3] = v.a;
}

void ko_cone_records(ko_ctx* c, float* o18) {
    for (uint32_t i = 0; i < c->n_cones; ++i) {
        const obj_t* o = &c->obj[c->n_tris + i];
        float r[18] = {o->base.x, o->base.y, o->base.z, o->r0, o->u.x, o->u.y, o->u.z, o->slope,
                       o->v.x, o->v.y, o->v.z, o->min_d, o->w.x, o->w.y, o->w.z, o->max_d, o->base_d, o->height};
        memcpy(o18 + 18 * (size_t)i, r, sizeof(r));
    }
}

void ko_tri_records(ko_ctx* c, float* o24, int32_t* lA) {
    for (uint32_t i = 0; i < c->n_tris; ++i) {
        const obj_t* o = &c->obj[i];
        v3 vv[8] = {o->A, o->B, o->C, o->ab, o->ac, o->na, o->nb, o->nc};
        for (int k = 0; k < 8; ++k) {
            o24[24 * (size_t)i + 3 * k] = vv[k].x;
            o24[24 * (size_t)i + 3 * k + 1] = vv[k].y;
            o24[24 * (size_t)i + 3 * k + 2] = vv[k].z;
        }
        if (lA) lA[i] = o->lA;
    }
}

uint32_t ko_bvh_nodes(ko_ctx* c, float* o6, int32_t* first, int32_t* count, int32_t* object_ids) {
    /* nodes are allocated in DFS preorder already (split allocates before recursing) */
    for (uint32_t i = 0; i < c->n_nodes; ++i) {
        const node_t* n = &c->nodes[i];
        if (o6) {
            float* d = o6 + 6 * (size_t)i;
            d[0] = n->box.mn.x; d[1] = n->box.mn.y; d[2] = n->box.mn.z;
            d[3] = n->box.mx.x; d[4] = n->box.mx.y; d[5] = n->box.mx.z;
        }
        if (first) first[i] = n->count ? n->first : -1;
        if (count) count[i] = n->count;
    }
    if (object_ids)
        for (uint32_t i = 0; i < c->n_obj; ++i) object_ids[i] = (int32_t)c->ids[i];
    return c->n_nodes;
}

uint32_t ko_bvh_depth(ko_ctx* c) { return c->depth; }

int ko_bsdf_sample(ko_ctx* c, int hit_obj, const khp_material* mat, const float in[3], const float n[3],
                   float sample_io[2], const float rng_hair[2], int flags_in, float out_dir[3], float* pdf, float f[3]) {
    shade_ctx_t s;
    s.obj = (hit_obj >= 0 && (uint32_t)hit_obj < c->n_obj) ? &c->obj[hit_obj] : &c->obj[0];
    s.m = mat;
    s.n = ld3(n);
    v3 out; int flags = flags_in, valid;
    float pd = 0.0f;
    v3 r = bsdf_sample(&s, ld3(in), s.n, sample_io, rng_hair, &out, &pd, &flags, &valid);
    out_dir[0] = out.x; out_dir[1] = out.y; out_dir[2] = out.z;
    *pdf = pd;
    f[0] = r.x; f[1] = r.y; f[2] = r.z;
    return flags;
}

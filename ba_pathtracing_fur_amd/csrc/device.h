// device.h -- gfx950 device functions of the hot path: BVH2 traversal,
// ray-cone / ray-triangle intersection, lights, BSDFs.  Each function states
// the KIRK lines it reproduces (paths relative to src/libraries/KIRK/).
// Float operation order follows GLM 0.9.9 / the KIRK source so results match
// the CPU restatement in oracle/ bit-for-bit (build: -ffp-contract=off).
#pragma once

#include <hip/hip_runtime.h>

#include "kmath.h"
#include "scene.h"

namespace khp {

constexpr float RAY_EPS_D = 1e-4f;   // KIRK::cRayEpsilon (Common/Ray.h:9)
constexpr float TRI_EPS_D = 1e-7f;   // cTriangleEpsilon (Common/Triangle.h:46)
constexpr int STACK_MAX = 64;        // >= BVH depth (checked on the host)

enum : int { F_TRANSPARENT = 1, F_SPECULAR = 2, F_EMISSIVE = 4, F_CYL_T = 8, F_CYL_TR = 16 };  // Bsdf.h:18-22

struct DevScene {
    const float4* __restrict__ prims;    // slot order, 4 x float4 per object
    const Aux* __restrict__ aux;         // slot order
    const float* __restrict__ tri_nrm;   // object-id order, 9 floats per triangle
    const float* __restrict__ tri_frame; // object-id order, 9 floats per triangle: hair frame u v w
    const DevNode* __restrict__ nodes;   // interior nodes
    const float4* __restrict__ wide;     // two-level records (traverse.h iterw), 8 float4 per node; null: not built
    const khp_material* __restrict__ mats;
    const DevLight* __restrict__ lights;
    int32_t n_lights;
    int32_t root_ref, root_cnt;
    float root_box[6];
    khp_environment env;
    khp_camera cam;
    // ABI 6 textures (null / 0 when the scene has none)
    const float* __restrict__ tri_uv;    // object-id order, 6 floats per triangle (reordered tca tcb tcc)
    const float* __restrict__ cone_h;    // cone order (object id - n_tris): Cylinder::m_height
    const DevTexture* __restrict__ tex;
    const uint8_t* __restrict__ texels;
    const DevMatTex* __restrict__ mtex;  // per material
    uint32_t n_tris;
    int32_t textured;
    khp_env_map env_map;
    const uint32_t* __restrict__ tri_slot;  // object-id order: the slot of each triangle (NaN-origin shadow rays)
    // khp_ctx_params.lds_nodes: the tree's top TOP_NODES interior records (BFS order) with
    // the refs between them rewritten to TOP_REF | index, and the root's ref in that form
    const float4* __restrict__ top;
    int32_t top_root;
};

// ---- textures (ABI 6) -------------------------------------------------------------------
// Texture::getColor (Texture.cpp:243-287): NaN -> red; a coordinate outside
// [0, 1] becomes pow(frac, wrap_mode) -- glm::pow resolves to std::pow(double,
// double) for the uchar mode, so TILE (1) gives the fraction and CLAMP (0)
// gives 1; then the nearest texel (int)(u * (w - 1)), channel expansion
// rrrr / rrrg / rgb1 / rgba and /255.  Texel indices are clamped into the
// image, where KIRK would read out of bounds (infinite coordinates).
__device__ __forceinline__ float tex_wrap(float x, uint32_t mode) {
    if (x > 1.0f || x < 0.0f) {
        const float f = x - floorf(x);
        if (mode == 1u) return f;
        if (mode == 0u) return 1.0f;
        return (float)pow((double)f, (double)mode);
    }
    return x;
}
__device__ __forceinline__ float4 tex_color(const DevScene& S, int32_t ti, float x, float y) {
    if (x != x || y != y) return make_float4(1.0f, 0.0f, 0.0f, 1.0f);  // Color::RED
    const DevTexture t = S.tex[ti];
    const float ux = tex_wrap(x, t.wrap), uy = tex_wrap(y, t.wrap);
    int sx = (int)(ux * (float)((int)t.w - 1)), sy = (int)(uy * (float)((int)t.h - 1));
    sx = sx < 0 ? 0 : (sx >= (int)t.w ? (int)t.w - 1 : sx);
    sy = sy < 0 ? 0 : (sy >= (int)t.h ? (int)t.h - 1 : sy);
    const uint8_t* p = S.texels + t.off + (size_t)t.ch * ((size_t)sy * t.w + (size_t)sx);
    const float r = p[0] / 255.0f;
    switch (t.ch) {
        case 4: return make_float4(r, p[1] / 255.0f, p[2] / 255.0f, p[3] / 255.0f);
        case 3: return make_float4(r, p[1] / 255.0f, p[2] / 255.0f, 1.0f);
        case 2: return make_float4(r, r, r, p[1] / 255.0f);
        default: return make_float4(r, r, r, r);
    }
}

// Material::getFromParam (Material.cpp:15-23) for every parameter the path
// tracer fetches: textured colours take the texel's rgb, textured roughness
// the length of its rgba (glm::length(vec4): sqrt((x*x + y*y) + (z*z + w*w))).
__device__ __forceinline__ void set_rgb(float* dst, float4 c) {
    dst[0] = c.x;
    dst[1] = c.y;
    dst[2] = c.z;
}
__device__ __forceinline__ void resolve_material(const DevScene& S, uint32_t mat, float tu, float tv,
                                                 khp_material& m) {
    const DevMatTex mt = S.mtex[mat];
    if (mt.t[MT_DIFFUSE] >= 0) set_rgb(m.diffuse, tex_color(S, mt.t[MT_DIFFUSE], tu, tv));
    if (mt.t[MT_SPECULAR] >= 0) set_rgb(m.specular, tex_color(S, mt.t[MT_SPECULAR], tu, tv));
    if (mt.t[MT_VOLUME] >= 0) set_rgb(m.volume, tex_color(S, mt.t[MT_VOLUME], tu, tv));
    if (mt.t[MT_EMISSION] >= 0) set_rgb(m.emission, tex_color(S, mt.t[MT_EMISSION], tu, tv));
    if (mt.t[MT_ROUGHNESS] >= 0) {
        const float4 c = tex_color(S, mt.t[MT_ROUGHNESS], tu, tv);
        m.roughness = sqrtf((c.x * c.x + c.y * c.y) + (c.z * c.z + c.w * c.w));
    }
}

// Environment::getColor (Environment.cpp:91-133).  Cube map: the face of the
// dominant axis (side = 1.5 -/+ 1.5 sign, the z faces with the opposite sign
// convention of KIRK's code), uv from the ratios as written there; sphere map:
// m = 2 sqrt(x^2 + y^2 + (z + 1)^2) with the z term in double, uv = d/m + 0.5.
__device__ __forceinline__ v3 env_color(const DevScene& S, v3 dir_in) {
    if (S.env_map.type == KHP_ENV_COLOR) return mk(S.env.color[0], S.env.color[1], S.env.color[2]);
    const v3 d = normalize(dir_in);
    float4 c;
    if (S.env_map.type == KHP_ENV_CUBE_MAP) {
        const float sx = (float)((0.0f < d.x) - (d.x < 0.0f)), sy = (float)((0.0f < d.y) - (d.y < 0.0f));
        const float sz = (float)((0.0f < d.z) - (d.z < 0.0f));
        const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
        const float mx = gmax(gmax(ax, ay), az);
        int side;
        float u, v;
        if (mx == ax) {
            side = (int)(0.0f + 1.5f - 1.5f * sx);
            u = (d.z / d.x + 1.0f) / 2.0f;
            v = (d.y / ax + 1.0f) / 2.0f;
        } else if (mx == ay) {
            side = (int)(1.0f + 1.5f - 1.5f * sy);
            u = (d.x / ay + 1.0f) / 2.0f;
            v = (d.z / d.y + 1.0f) / 2.0f;
        } else {
            side = (int)(2.0f + 1.5f + 1.5f * sz);
            u = -(d.x / d.z + 1.0f) / 2.0f;
            v = (d.y / az + 1.0f) / 2.0f;
        }
        c = tex_color(S, S.env_map.tex[side], u, v);
    } else {
        const double zz = (double)d.z + 1.0;
        const float m = (float)(2.0 * sqrt((double)(d.x * d.x + d.y * d.y) + zz * zz));
        const float u = (float)((double)(d.x / m) + 0.5), v = (float)((double)(d.y / m) + 0.5);
        c = tex_color(S, S.env_map.tex[0], u, v);
    }
    return mk(c.x, c.y, c.z);
}

struct Ray {
    v3 o, d;
};
// KIRK::Ray ctor normalises (Common/Ray.cpp:11-15)
__device__ __forceinline__ Ray make_ray(v3 o, v3 d) {
    Ray r;
    r.o = o;
    r.d = normalize(d);
    return r;
}
__device__ __forceinline__ v3 follow(const Ray& r, float t) { return r.d * t + r.o; }

// BoundingVolume::intersects (CPU_Datastructures/BoundingBox.cpp:142-194)
__device__ __forceinline__ bool slab(float mnx, float mny, float mnz, float mxx, float mxy, float mxz, const Ray& r,
                                     v3 inv, float& t0, float& t1) {
    // dir_sign = dir < 0 (CPU_BVH.cpp:55-56); taken from the direction, not from inv (-0.0)
    const bool sgn[3] = {r.d.x < 0.0f, r.d.y < 0.0f, r.d.z < 0.0f};
    float tmin = ((sgn[0] ? mxx : mnx) - r.o.x) * inv.x;
    float tmax = ((sgn[0] ? mnx : mxx) - r.o.x) * inv.x;
    float tymin = ((sgn[1] ? mxy : mny) - r.o.y) * inv.y;
    float tymax = ((sgn[1] ? mny : mxy) - r.o.y) * inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = ((sgn[2] ? mxz : mnz) - r.o.z) * inv.z;
    float tzmax = ((sgn[2] ? mnz : mxz) - r.o.z) * inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    t0 = tmin;
    t1 = tmax;
    return true;
}

__device__ __forceinline__ bool is_tri(float4 r0) { return bits_from_f(r0.w) == TRI_TAG; }

// Triangle::closestIntersection / isIntersection (Common/Triangle.cpp:152-184, 213-242)
__device__ __forceinline__ bool tri_test(float4 r0, float4 r1, float4 r2, const Ray& r, float tMin, float tMax,
                                         float& t, float& u, float& v) {
    v3 A = mk(r0.x, r0.y, r0.z), ab = mk(r1.x, r1.y, r1.z), ac = mk(r2.x, r2.y, r2.z);
    v3 dv = cross(r.d, ac);
    float det = dot(dv, ab);
    if (fabsf(det) < TRI_EPS_D) return false;
    float inv = 1.0f / det;
    v3 w = r.o - A;
    u = dot(dv, w) * inv;
    if (u < 0.0f || u > 1.0f) return false;
    v3 wu = cross(w, ab);
    v = dot(wu, r.d) * inv;
    if (v < 0.0f || u + v > 1.0f) return false;
    t = dot(wu, ac) * inv;
    if ((t < tMin) || (t > tMax)) return false;
    return true;
}

// The barycentrics tri_test computes for an accepted triangle (the same
// operations; they depend on the ray and the triangle only, not on the
// window).  The closest-hit traversal keeps only t and the slot; the shading
// side recomputes u, v from the ray it already has (triangles; cones: 0, 0).
__device__ __forceinline__ void tri_uv(float4 r0, float4 r1, float4 r2, const Ray& r, float& u, float& v) {
    v3 A = mk(r0.x, r0.y, r0.z), ab = mk(r1.x, r1.y, r1.z), ac = mk(r2.x, r2.y, r2.z);
    v3 dv = cross(r.d, ac);
    float det = dot(dv, ab);
    float inv = 1.0f / det;
    v3 w = r.o - A;
    u = dot(dv, w) * inv;
    v3 wu = cross(w, ab);
    v = dot(wu, r.d) * inv;
}

// Cylinder::closestIntersection (Common/Cylinder.cpp:73-156) and
// Cylinder::isIntersection (:158-228), open cone frustum.  The two differ only
// in the quadratic's leading coefficient -- a = 1 - Dy^2 (1 + s^2) for the
// closest hit, a = Dx^2 + Dz^2 - s^2 Dy^2 for the any hit -- and in the any
// hit's fixed tMin = 0; everything after a is the same sequence.  any_form
// selects a (a compile-time constant in cone_closest / cone_any; a per-lane
// value in the path kernel's mixed closest/any traversal, where both
// coefficients are computed by their own expressions and one is selected).
__device__ __forceinline__ bool cone_quadratic(float4 c0, float4 c1, float4 c2, float4 c3, const Ray& r, bool any_form,
                                               float tMin, float tMax, float& t) {
    v3 base = mk(c0.x, c0.y, c0.z), U = mk(c1.x, c1.y, c1.z), Vv = mk(c2.x, c2.y, c2.z), W = mk(c3.x, c3.y, c3.z);
    float r0 = c0.w, slope = c1.w, min_d = c2.w, max_d = c3.w;
    v3 P = r.o - base;
    P = mk(dot(P, U), dot(P, Vv), dot(P, W));
    v3 D = mk(dot(r.d, U), dot(r.d, Vv), dot(r.d, W));
    const float a_closest = 1.0f - D.y * D.y * (1.0f + slope * slope);
    const float a_any = D.x * D.x + D.z * D.z - slope * slope * D.y * D.y;
    float a = any_form ? a_any : a_closest;
    float b = P.x * D.x + P.z * D.z + r0 * slope * D.y - slope * slope * P.y * D.y;
    float c = r0 - slope * P.y;
    c = P.x * P.x + P.z * P.z - c * c;
    float disc = b * b - a * c;
    if (disc < 0.0f) return false;
    disc = sqrtf(disc);
    float t1 = (-b - disc) / a;
    float t2 = (-b + disc) / a;
    if ((t2 < tMin) || (t1 > tMax)) return false;
    if (t1 < RAY_EPS_D) {
        if ((t2 > tMax) || (t2 < tMin)) return false;
        float d = dot(Vv, follow(r, t2));
        if (d >= min_d && d <= max_d) { t = t2; return true; }
        return false;
    }
    if ((t1 < tMin) && (t2 > tMax)) return false;
    float d = dot(Vv, follow(r, t1));
    if (d >= min_d && d <= max_d) { t = t1; return true; }
    d = dot(Vv, follow(r, t2));
    if (d >= min_d && d <= max_d) { t = t2; return true; }
    return false;
}

__device__ __forceinline__ bool cone_closest(float4 c0, float4 c1, float4 c2, float4 c3, const Ray& r, float tMin,
                                             float tMax, float& t) {
    return cone_quadratic(c0, c1, c2, c3, r, false, tMin, tMax, t);
}

// Cylinder::isIntersection (Common/Cylinder.cpp:158-228): note a = Dx^2+Dz^2-s^2 Dy^2.
__device__ __forceinline__ bool cone_any(float4 c0, float4 c1, float4 c2, float4 c3, const Ray& r, float tMax) {
    float t;
    return cone_quadratic(c0, c1, c2, c3, r, true, 0.0f, tMax, t);
}

#include "traverse.h"

// ---------------------------------------------------------------------------
// lights (Common/Light.h, Common/Light.cpp)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float dist_att(const DevLight& L, float d) {  // Light.h:70-73
    return (L.c > 0.0f || (L.l > 0.0f && L.q > 0.0f)) ? 1.0f / ((L.c + L.l * d) + L.q * (d * d)) : 1.0f;
}
__device__ __forceinline__ v3 uniform_sphere(float u0, float u1) {  // Light.cpp:66-72 (m_dist is double)
    float phi = (float)((double)u0 * 2.0 * M_PI_D);
    float ct = (float)(2.0 * (double)u1 - 1.0);
    float st = sqrtf(gmax(0.0f, 1.0f - ct * ct));
    return mk(st * k_cosf(phi), st * k_sinf(phi), ct);
}
__device__ __forceinline__ void ortho_base(v3 n, v3& s, v3& t) {  // Light.cpp:112-118
    if (fabsf(n.x) > fabsf(n.y)) s = mk(-n.z, 0.0f, n.x) / sqrtf(n.x * n.x + n.z * n.z);
    else s = mk(0.0f, n.z, -n.y) / sqrtf(n.y * n.y + n.z * n.z);
    t = cross(n, s);
}
// calcLightdir, randomize = true (Light.cpp:127-145, 278-296, 327-343, 463-475)
__device__ __forceinline__ Ray light_dir(const DevLight& L, v3 p, float u0, float u1, float& att) {
    if (L.kind == KHP_LIGHT_POINT) {
        v3 pos = ld3(L.position);
        v3 direction = normalize(pos - p);
        v3 pt = uniform_sphere(u0, u1);
        pos = pos + pt * L.radius;
        float dd = gclamp(dot(pt, -direction), 0.0f, 1.0f);
        float dist = length(pos - p);
        att = dd * dist_att(L, dist);
        return make_ray(p, pos - p);
    }
    if (L.kind == KHP_LIGHT_QUAD) {
        v3 v0 = ld3(L.vert[0]), v1 = ld3(L.vert[1]), v2 = ld3(L.vert[2]), v3_ = ld3(L.vert[3]);
        v3 x1 = v0 + (v1 - v0) * u0;
        v3 x2 = v3_ + (v2 - v3_) * u0;
        v3 ip = x1 + (x2 - x1) * u1;
        v3 ld = ip - p;
        float dd = gclamp(dot(normalize(-ld), ld3(L.direction)), 0.0f, 1.0f);
        att = dd * dist_att(L, length(ld));
        return make_ray(p, ld);
    }
    if (L.kind == KHP_LIGHT_SPOT) {
        float rr = sqrtf(u0);
        float th = (float)(2.0 * M_PI_D * (double)u1);
        float x = rr * k_cosf(th), y = rr * k_sinf(th);
        v3 d = mk(L.radius * x, L.radius * y, 0.0f);
        v3 s, t;
        ortho_base(ld3(L.direction), s, t);
        v3 pt = s * d.x + t * d.y;
        v3 ld = (ld3(L.position) + pt) - p;
        float ang = k_acosf(dot(normalize(-ld), ld3(L.direction))) * RAD2DEG;
        float delta = 1.0f - gclamp((ang - L.inner) / (L.outer - L.inner), 0.0f, 1.0f);
        delta = delta * delta * delta * delta;
        att = delta * dist_att(L, length(ld));
        return make_ray(p, ld);
    }
    v3 pt = uniform_sphere(u0, u1) * L.radius;
    pt = pt - ld3(L.direction);
    v3 dn = normalize(pt);
    v3 pos = dn * 1e16f;
    att = 1.0f;
    return make_ray(p, pos - p);
}
__device__ __forceinline__ bool light_tri(const Ray& r, v3 v1, v3 v2, v3 v3_, float& t) {  // Light.cpp:13-64
    v3 e1 = v2 - v1, e2 = v3_ - v1;
    v3 P = cross(r.d, e2);
    float det = dot(e1, P);
    if (det > -FLT_EPS_ && det < FLT_EPS_) return false;
    float inv = 1.0f / det;
    v3 T = r.o - v1;
    float u = dot(T, P) * inv;
    if (u < 0.0f || u > 1.0f) return false;
    v3 Q = cross(T, e1);
    float v = dot(r.d, Q) * inv;
    if (v < 0.0f || u + v > 1.0f) return false;
    t = dot(e2, Q) * inv;
    return t > FLT_EPS_;
}
// isIntersection (Light.cpp:169-189, 227-232, 367-428, 497-501)
__device__ __forceinline__ bool light_isect(const DevLight& L, const Ray& r, float& t) {
    if (L.kind == KHP_LIGHT_POINT) {
        float rsq = L.radius * L.radius;
        if (rsq == 0.0f) return false;
        v3 pos = ld3(L.position);
        if (dot(r.d, r.o - pos) > 0.0f) return false;
        float a = dot(r.d, r.d);
        float b = dot(r.d, (r.o - pos) * 2.0f);
        float c = ((dot(pos, pos) + dot(r.o, r.o)) - 2.0f * dot(r.o, pos)) - rsq;
        float d = b * b - 4.0f * a * c;
        if (d < 0.0f) return false;
        d = sqrtf(d);
        t = (-0.5f) * (b + d) / a;
        return true;
    }
    if (L.kind == KHP_LIGHT_QUAD) {
        v3 v0 = ld3(L.vert[0]), v1 = ld3(L.vert[1]), v2 = ld3(L.vert[2]), v3_ = ld3(L.vert[3]);
        return light_tri(r, v0, v1, v3_, t) || light_tri(r, v2, v3_, v1, t);
    }
    if (L.kind == KHP_LIGHT_SPOT) {
        if (L.radius == 0.0f) return false;
        v3 n = ld3(L.direction), x;
        if (fabsf(n.x) > fabsf(n.y)) x = mk(-n.z, 0.0f, n.x) / sqrtf(n.x * n.x + n.z * n.z);
        else x = mk(0.0f, n.z, -n.y) / sqrtf(n.y * n.y + n.z * n.z);
        v3 y = cross(n, x);
        v3 v1 = ld3(L.position), v2 = v1 + x, v3_ = v1 + y;
        v3 e1 = v2 - v1, e2 = v3_ - v1;
        v3 P = cross(r.d, e2);
        float det = dot(e1, P);
        if (det > -FLT_EPS_ && det < FLT_EPS_) return false;
        float inv = 1.0f / det;
        v3 T = r.o - v1;
        float u = dot(T, P) * inv;
        v3 Q = cross(T, e1);
        float v = dot(r.d, Q) * inv;
        if (u * u + v * v > L.radius * L.radius) return false;
        t = dot(e2, Q) * inv;
        return t > FLT_EPS_;
    }
    return false;
}
// sampleLightSource (Light.cpp:196-199, 234-239, 436-440, 508-511)
__device__ __forceinline__ v3 light_emit(const DevLight& L, v3 dir) {
    float cdiv = L.c > 0.0f ? L.c : 1.0f;
    v3 col = ld3(L.color);
    if (L.kind == KHP_LIGHT_POINT) return (col * ONE_OVER_PI) / cdiv;
    if (L.kind == KHP_LIGHT_QUAD || L.kind == KHP_LIGHT_SPOT) {
        float dd = dot(normalize(-dir), ld3(L.direction)) < 0.0f ? 0.0f : 1.0f;
        return (col * (ONE_OVER_PI * dd)) / cdiv;
    }
    return col;
}

// ---------------------------------------------------------------------------
// BSDFs (Common/Shading/Bsdf.cpp)
// ---------------------------------------------------------------------------
__device__ __forceinline__ float fresnel_dielectric(float cos_theta, float eta_i, float eta_t) {  // :143-171
    float ci = gclamp(cos_theta, -1.0f, 1.0f);
    if (ci <= 0.0f) {
        float t = eta_i;
        eta_i = eta_t;
        eta_t = t;
        ci = fabsf(ci);
    }
    float si = sqrtf(gmax(0.0f, 1.0f - ci * ci));
    float st = eta_i / eta_t * si;
    if (st >= 1.0f) return 1.0f;
    float ct = sqrtf(gmax(0.0f, 1.0f - st * st));
    float rparl = ((eta_t * ci) - (eta_i * ct)) / ((eta_t * ci) + (eta_i * ct));
    float rperp = ((eta_i * ci) - (eta_t * ct)) / ((eta_i * ci) + (eta_t * ct));
    return (rparl * rparl + rperp * rperp) / 2.0f;
}
__device__ __forceinline__ v3 cosine_hemi(float u0, float u1) {  // :95-132
    float ox = 2.0f * u0 - 1.0f, oy = 2.0f * u1 - 1.0f, dx, dy;
    if (ox == 0.0f && oy == 0.0f) {
        dx = 0.0f;
        dy = 0.0f;
    } else {
        float th, r;
        if (fabsf(ox) > fabsf(oy)) { r = ox; th = QUARTER_PI * (oy / ox); }
        else { r = oy; th = HALF_PI - QUARTER_PI * (ox / oy); }
        dx = r * k_cosf(th);
        dy = r * k_sinf(th);
    }
    return mk(dx, dy, sqrtf(gmax(0.0f, 1.0f - dx * dx - dy * dy)));
}
__device__ __forceinline__ v3 sample_angle(float u0, float u1, float max_angle) {  // :117-123
    float phi = (float)((double)(u0 * 2.0f) * M_PI_D);
    float ct = 1.0f - u1 * (1.0f - k_cosf(max_angle));
    float st = sqrtf(1.0f - ct * ct);
    return mk(k_cosf(phi) * st, k_sinf(phi) * st, ct);
}
__device__ __forceinline__ float normal_gauss_pdf(float x, float mean, float sd) {  // :79-85
    const float inv_sqrt_2pi = 0.3989422804014327f;
    float a = (x - mean) / sd;
    return inv_sqrt_2pi / sd * k_expf(-0.5f * a * a);
}

struct ShadeCtx {
    const khp_material* m;
    v3 n;
    v3 U, V, W;   // hair frame (Object::getU/V/W): the cone's, or the fiber's for fur triangles
};

// BSDF::evaluateLight dispatch (Bsdf.cpp:197-202, 310-318, 771-776; others 0)
__device__ __forceinline__ v3 bsdf_eval(const ShadeCtx& s, v3 in, v3 out) {
    int kind = s.m->bsdf;
    bool refl = dot(in, s.n) * dot(out, s.n) > 0.0f;
    v3 diff = mk(s.m->diffuse[0], s.m->diffuse[1], s.m->diffuse[2]);
    if (kind == KHP_BSDF_LAMBERTIAN_REFLECTION || kind == KHP_BSDF_MARSCHNER_HAIR)
        return refl ? diff * ONE_OVER_PI : mk(0.0f, 0.0f, 0.0f);
    if (kind == KHP_BSDF_LAMBERTIAN_TRANSMISSION) return !refl ? diff * ONE_OVER_PI : mk(0.0f, 0.0f, 0.0f);
    return mk(0.0f, 0.0f, 0.0f);
}

// Hair R lobes: Marschner (Bsdf.cpp:465-489, 669-736) and d'Eon (:784-808, 969-1017).
// TT/TRT are unreachable (p = 0 hard-coded, :669/:969).
template <bool DEON>
__device__ __forceinline__ v3 hair_r(const ShadeCtx& s, v3 in, v3 n, float sample[2], float h0, float h1, v3& out,
                                     float& pdf, int& flags) {
    float ior = s.m->ior;
    v3 nin = normalize(in);
    v3 in_cyl = world_to_local(in, s.V, s.U, s.W);
    if ((flags & F_CYL_T) || (flags & F_CYL_TR)) {
        out = mk(0.0f, 0.0f, 1.0f);
        return mk(0.0f, 0.0f, 0.0f);
    }
    float alpha, beta;
    if (DEON) {
        alpha = (-1.0f * (5.0f + 5.0f * h0)) * DEG2RAD;
        beta = (5.0f + 5.0f * h1) * DEG2RAD;
    } else {
        alpha = -1.0f * (5.0f + 5.0f * h0);
        beta = 5.0f + 5.0f * h1;
    }
    v3 o1 = reflect(-nin, faceforward(n, -nin, n));
    o1 = rotate_rowvec(o1, alpha, s.V);
    flags = F_SPECULAR;
    v3 oc = world_to_local(o1, s.V, s.U, s.W);
    float ti = k_atan2f(k_hypotf(in_cyl.x, in_cyl.z), in_cyl.y);
    float tr = k_atan2f(k_hypotf(oc.x, oc.z), oc.y);
    out = o1;
    if (!DEON) {
        float th = (tr + ti) / 2.0f;
        float td = (tr - ti) / 2.0f;
        float gx = th - alpha;
        sample[0] = ti;
        sample[1] = 0.0f;
        pdf = normal_gauss_pdf(gx, 0.0f, beta);
        float gi = angle(nin, normalize(n));
        float h = k_sinf(gi);
        float dh = fabsf(-2.0f / sqrtf(1.0f - h * h));
        float cgi = k_cosf(gi);
        float sgi = k_sinf(gi);
        float x1 = sqrtf(ior * ior - sgi * sgi);
        float b1 = x1 / cgi;
        float b2 = ior * ior * cgi / x1;
        float F = fresnel_dielectric(gi, b1, b2);
        float nr = 0.5f * F * dh;
        float ctd = k_cosf(td);
        float sc = pdf * nr / (ctd * ctd);
        return mk(sc, sc, sc);
    } else {
        float v = beta * beta;
        float csch = 1.0f / k_sinhf((1.0f / v) * DEG2RAD);
        float dv = v * RAD2DEG;
        float e = k_expf((k_sinf(-ti) * k_sinf(tr)) / dv);
        float bes = (float)k_j0((double)((k_cosf(-ti) * k_cosf(tr)) / dv));
        pdf = (csch / (2.0f * v)) * e * bes;
        float pi_ = k_atan2f(in_cyl.x, in_cyl.y);
        float pr = k_atan2f(oc.x, oc.y);
        float dr = 0.25f * fabsf(k_cosf(pr - pi_ / 2.0f));
        float F = fresnel_dielectric(0.5f * k_acosf(dot(nin, normalize(o1))), 1.0f, ior);
        float nr = 0.5f * F * dr;
        float r = pdf * nr;
        return mk(r, r, r);
    }
}

// BSDF::sample (Bsdf.cpp:179-184) + localSample dispatch; valid=false on the
// `dot(ray_in, normal) == 0` early exit.
// Inlined into k_shade: measured 2.02 -> 1.66 ms per frame against a real call
// (whose frame spilled 41 SGPRs and 112 B of scratch), +0.7% at the metric row
// (profiles/r02p_bsdf_inline.json).
// KINDS: the BSDF kinds the scene's materials use (bit k = khp_bsdf_kind k), a
// compile-time set: the other cases are compiled out (their registers with
// them).  The host instantiates a kernel whose set covers every material.
template <uint32_t KINDS = 0xFFFFFFFFu>
__device__ __forceinline__
v3 bsdf_sample(const ShadeCtx& s, v3 in, v3 n, float sample[2], float h0, float h1, v3& out,
                                       float& pdf, int& flags, bool& valid) {
    v3 zero = mk(0.0f, 0.0f, 0.0f);
    valid = true;
    if (dot(in, n) == 0.0f) {
        valid = false;
        out = mk(0.0f, 0.0f, 1.0f);
        return zero;
    }
    const khp_material* m = s.m;
    v3 diff = mk(m->diffuse[0], m->diffuse[1], m->diffuse[2]);
    v3 spec = mk(m->specular[0], m->specular[1], m->specular[2]);
    v3 vol = mk(m->volume[0], m->volume[1], m->volume[2]);
    switch (m->bsdf) {
        case KHP_BSDF_LAMBERTIAN_REFLECTION: {  // :186-195
            if constexpr (!(KINDS & (1u << KHP_BSDF_LAMBERTIAN_REFLECTION))) __builtin_unreachable();
            bool entering = dot(in, n) > 0.0f;
            v3 h = cosine_hemi(sample[0], sample[1]);
            out = local_to_world_normal(entering ? h : -h, n);
            pdf = fabsf(dot(out, n)) * ONE_OVER_PI;
            flags = 0;
            if (pdf == 0.0f) return zero;
            return diff * ONE_OVER_PI;
        }
        case KHP_BSDF_SPECULAR_REFLECTION: {  // :210-217
            if constexpr (!(KINDS & (1u << KHP_BSDF_SPECULAR_REFLECTION))) __builtin_unreachable();
            out = reflect(-in, faceforward(n, -in, n));
            pdf = 1.0f;
            flags |= F_SPECULAR;
            return spec / fabsf(dot(out, n));
        }
        case KHP_BSDF_GLOSSY: {  // :227-245
            if constexpr (!(KINDS & (1u << KHP_BSDF_GLOSSY))) __builtin_unreachable();
            float rad = (180.0f - (1.0f - m->roughness) * 180.0f) * DEG2RAD;
            v3 refl = reflect(-in, faceforward(n, -in, n));
            v3 sp = sample_angle(sample[0], sample[1], rad);
            out = local_to_world_normal(sp, refl);
            if (dot(out, faceforward(n, -in, n)) < 0.0f) out = local_to_world_normal(sp * mk(-1.0f, -1.0f, 1.0f), refl);
            pdf = 1.0f;
            flags |= F_SPECULAR;
            return spec / fabsf(dot(out, n));
        }
        case KHP_BSDF_SPECULAR_TRANSMISSION: {  // :258-288
            if constexpr (!(KINDS & (1u << KHP_BSDF_SPECULAR_TRANSMISSION))) __builtin_unreachable();
            bool entering = dot(in, n) > 0.0f;
            float ei = entering ? 1.0f : m->ior, et = entering ? m->ior : 1.0f;
            float F = fresnel_dielectric(fabsf(dot(in, n)), ei, et);
            flags |= F_SPECULAR;
            out = refract(normalize(-in), faceforward(n, -in, n), ei / et);
            pdf = 1.0f;
            if (!is_zero(out) && !k_isnan(out.x)) {
                flags |= F_TRANSPARENT;
                v3 ft = vol * (1.0f - F);
                ft = ft * ((ei * ei) / (et * et));
                return ft / fabsf(dot(out, n));
            }
            return zero;
        }
        case KHP_BSDF_LAMBERTIAN_TRANSMISSION: {  // :298-308
            if constexpr (!(KINDS & (1u << KHP_BSDF_LAMBERTIAN_TRANSMISSION))) __builtin_unreachable();
            bool entering = dot(in, n) > 0.0f;
            v3 h = cosine_hemi(sample[0], sample[1]);
            out = local_to_world_normal(entering ? -h : h, n);
            pdf = fabsf(dot(out, n)) * ONE_OVER_PI;
            flags = F_TRANSPARENT;
            if (pdf == 0.0f) return zero;
            return vol * ONE_OVER_PI;
        }
        case KHP_BSDF_GLASS: {  // :326-357
            if constexpr (!(KINDS & (1u << KHP_BSDF_GLASS))) __builtin_unreachable();
            bool entering = dot(in, n) > 0.0f;
            float ei = entering ? 1.0f : m->ior, et = entering ? m->ior : 1.0f;
            float F = fresnel_dielectric(fabsf(dot(normalize(in), n)), ei, et);
            flags |= F_SPECULAR;
            v3 nin = normalize(in);
            out = refract(normalize(-in), faceforward(n, -nin, n), ei / et);
            if (!is_zero(out) && sample[1] > F && !k_isnan(out.x)) {
                flags |= F_TRANSPARENT;
                pdf = 1.0f - F;
                v3 ft = vol * (1.0f - F);
                ft = ft * ((ei * ei) / (et * et));
                return ft / fabsf(dot(out, n));
            }
            out = reflect(normalize(-in), faceforward(n, -nin, n));
            pdf = F;
            return (spec * F) / fabsf(dot(out, n));
        }
        case KHP_BSDF_MILK_GLASS: {  // :367-416
            if constexpr (!(KINDS & (1u << KHP_BSDF_MILK_GLASS))) __builtin_unreachable();
            bool entering = dot(in, n) > 0.0f;
            float ei = entering ? 1.0f : m->ior, et = entering ? m->ior : 1.0f;
            v3 nin = normalize(in);
            float F = fresnel_dielectric(fabsf(dot(nin, n)), ei, et);
            flags |= F_SPECULAR;
            v3 refr = refract(normalize(-in), faceforward(n, -nin, n), ei / et);
            float rad = (180.0f - (1.0f - m->roughness) * 180.0f) * DEG2RAD;
            if (!is_zero(refr) && sample[1] > F && !k_isnan(refr.x)) {
                v3 sp = sample_angle(sample[0], sample[1], rad);
                out = local_to_world_normal(sp, refr);
                if (dot(out, faceforward(n, -in, n)) > 0.0f)
                    out = local_to_world_normal(sp * mk(-1.0f, -1.0f, 1.0f), refr);
                flags |= F_TRANSPARENT;
                pdf = 1.0f - F;
                v3 ft = vol * (1.0f - F);
                ft = ft * ((ei * ei) / (et * et));
                return ft / fabsf(dot(out, n));
            }
            v3 refl = reflect(-in, faceforward(n, -in, n));
            v3 sp = sample_angle(sample[0], sample[1], rad);
            out = local_to_world_normal(sp, refl);
            if (dot(out, faceforward(n, -in, n)) < 0.0f) out = local_to_world_normal(sp * mk(-1.0f, -1.0f, 1.0f), refl);
            pdf = F;
            return (spec * F) / fabsf(dot(out, n));
        }
        case KHP_BSDF_EMISSION:  // :427-435
            if constexpr (!(KINDS & (1u << KHP_BSDF_EMISSION))) __builtin_unreachable();
            pdf = 1.0f;
            out = zero;
            flags = F_EMISSIVE;
            return mk(1.0f, 1.0f, 1.0f);
        case KHP_BSDF_TRANSPARENT:  // :445-454
            if constexpr (!(KINDS & (1u << KHP_BSDF_TRANSPARENT))) __builtin_unreachable();
            out = -in;
            flags = F_TRANSPARENT | F_SPECULAR;
            pdf = 1.0f;
            return vol / fabsf(dot(out, n));
        case KHP_BSDF_MARSCHNER_HAIR:
            if constexpr (!(KINDS & (1u << KHP_BSDF_MARSCHNER_HAIR))) __builtin_unreachable();
            return hair_r<false>(s, in, n, sample, h0, h1, out, pdf, flags);
        case KHP_BSDF_DEON_HAIR:
            if constexpr (!(KINDS & (1u << KHP_BSDF_DEON_HAIR))) __builtin_unreachable();
            return hair_r<true>(s, in, n, sample, h0, h1, out, pdf, flags);
        default:
            out = mk(0.0f, 0.0f, 1.0f);
            pdf = 0.0f;
            return zero;
    }
}

}  // namespace khp

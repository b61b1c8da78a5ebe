// lightpath.h -- the light-path (bidirectional) variant of KIRK's GLSL path
// tracer, SURVEY §8(f)4 (khp_bdpt_params, ABI 7).
//
// lbb_construction.compute:195-403 traces light subpaths (generatePrimaryLightRays,
// traceLightRays, shadeLightRays); pt_shade.compute:146-201 connects each
// camera hit to the vertices of one randomly chosen subpath in place of the
// next-event estimate.  Here a subpath is one thread of k_light_paths (a few
// hundred thousand short paths per batch, next to hundreds of millions of
// camera paths), and the connections are shadow records of the wavefront
// (k_shade emits them as one contiguous group per path, k_shadow traces them,
// k_shadow_finish adds a group's unoccluded contributions in vertex order).
// The arithmetic is oracle/kirk_oracle.c's light_subpath / bdpt_connect.
#pragma once
// (included from render.hip after device.h, inside no namespace)

namespace khp {

constexpr float GL_PI = 3.14159265359f;           // inc_random.compute:11 (a GLSL float)
constexpr float GL_ONE_OVER_PI = 0.31830988618f;  // inc_random.compute:12
constexpr float GL_DEG2RAD = 0.01745329251994329577f;
constexpr uint32_t LPATH_SEED = 0x4C504154u;      // light-path RNG: path_key(seed ^ LPATH_SEED, s * L + light, k)

constexpr uint32_t IMG_BOUNCE = 4095u;            // draw dims of the image-plane pass: bounce slot 4095

struct BdptDev {
    uint32_t on, Ns, L, J;
    float bias, bounce_bias, min_pdf;
    uint32_t img;      // shadeBDPTImagePlane pass on
    const float4* lv;  // [sample slot][Ns][L][J] x 3 float4: (pos, valid) (din, 0) (hit colour, 0)
};

// cosineHemisphereSample / uniformSphereSample / sampleAngle (inc_random.compute:50-81)
__device__ __forceinline__ v3 gl_cos_hemi(float u, float v) {
    const float r = sqrtf(u), th = 2.0f * GL_PI * v;
    const float x = r * k_cosf(th), y = r * k_sinf(th);
    return mk(x, y, sqrtf(gmax(0.0f, (1.0f - x * x) - y * y)));
}
__device__ __forceinline__ v3 gl_uniform_sphere(float u, float v) {
    const float phi = v * 2.0f * GL_PI, ct = 2.0f * u - 1.0f;
    const float st = sqrtf(gmax(0.0f, 1.0f - ct * ct));
    return mk(st * k_cosf(phi), st * k_sinf(phi), ct);
}
__device__ __forceinline__ v3 gl_sample_angle(float u, float v, float max_angle) {
    const float phi = v * 2.0f * GL_PI, ct = 1.0f - u * (1.0f - k_cosf(max_angle));
    const float st = sqrtf(1.0f - ct * ct);
    return mk(k_cosf(phi) * st, k_sinf(phi) * st, ct);
}
// the (s, t, n) frame of lbb_construction.compute:42-45 and localToWorld (BSDF/header.compute:23-26)
__device__ __forceinline__ v3 gl_to_world(v3 v, v3 n) {
    const v3 s = normalize(n.y * n.y > n.x * n.x ? mk(0.0f, n.z, -n.y) : mk(-n.z, 0.0f, n.x));
    const v3 t = normalize(cross(n, s));
    return (s * v.x + t * v.y) + n * v.z;
}
// calcLightBounce{Point,Sun,Spot,Quad} (lbb_construction.compute:35-141): the ray leaving the light
__device__ __forceinline__ Ray gl_light_ray(const DevLight& L, float a0, float a1, float b0, float b1) {
    Ray r;
    if (L.kind == KHP_LIGHT_POINT) {
        const v3 n = gl_uniform_sphere(a0, a1);
        r.o = ld3(L.position) + n * L.radius;
        r.d = gl_to_world(gl_cos_hemi(b0, b1), n);
    } else if (L.kind == KHP_LIGHT_SUN) {
        const v3 pos = -ld3(L.direction) + gl_uniform_sphere(a0, a1) * L.radius;
        const v3 dn = normalize(pos);
        r.o = pos + dn * 1e16f;
        r.d = ld3(L.direction);
    } else if (L.kind == KHP_LIGHT_SPOT) {
        v3 pr = gl_cos_hemi(a0, a1);
        pr.z = 0.0f;
        pr = pr * L.radius;
        const v3 dr = gl_sample_angle(b0, b1, L.outer * GL_DEG2RAD);
        r.o = ld3(L.position) + gl_to_world(pr, ld3(L.direction));
        r.d = gl_to_world(dr, ld3(L.direction));
    } else {
        const v3 v0 = ld3(L.vert[0]), v1 = ld3(L.vert[1]), v2 = ld3(L.vert[2]), v3_ = ld3(L.vert[3]);
        const v3 x1 = v0 + (v1 - v0) * a0;
        const v3 x2 = v3_ + (v2 - v3_) * a0;
        r.o = x1 + (x2 - x1) * a1;
        r.d = gl_to_world(gl_cos_hemi(b0, b1), ld3(L.direction));
    }
    r.d = normalize(r.d);
    return r;
}
// angularAttenuation (inc_light.compute:207-237)
__device__ __forceinline__ float gl_ang_att(const DevLight& L, v3 d) {
    if (L.kind == KHP_LIGHT_SPOT) {
        const float ang = k_acosf(dot(normalize(-d), ld3(L.direction))) * RAD2DEG;
        return 1.0f - gclamp((ang - L.inner) / (L.outer - L.inner), 0.0f, 1.0f);
    }
    if (L.kind == KHP_LIGHT_QUAD) return dot(normalize(-d), ld3(L.direction));
    return 1.0f;
}

}  // namespace khp

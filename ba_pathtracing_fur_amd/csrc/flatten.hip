// flatten.hip -- CPU::Scene::flattenNode's per-object work on the device
// (SURVEY §8(f)2): the Triangle / Cylinder ctor state of every object, and the
// seeded hairball (Mesh::addFurToFaces recurrence + the fiber -> cone rule of
// CPU_Scene.cpp:121-144) generated straight into HBM.  The arithmetic is
// objects.h, the same source the host flatten (scene.cpp) runs.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "device_build.h"
#include "objects.h"

namespace khp {
namespace fl {

__global__ void k_flatten_tris(const float* __restrict__ tv, const float* __restrict__ tn,
                               const uint32_t* __restrict__ tm, const float* __restrict__ uv_in, uint32_t n_tris,
                               uint32_t n_mat, float4* rec, Aux* aux, float* bounds, float* cen, float* nrm,
                               float* uv_out, uint32_t* err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_tris) return;
    const float* v = tv + 9 * (size_t)i;
    const float* n = tn + 9 * (size_t)i;
    float r[16];
    tri_object(ld3(v), ld3(v + 3), ld3(v + 6), ld3(n), ld3(n + 3), ld3(n + 6), r, bounds + 6 * (size_t)i,
               cen + 3 * (size_t)i, nrm + 9 * (size_t)i, uv_in ? uv_in + 6 * (size_t)i : nullptr,
               uv_out ? uv_out + 6 * (size_t)i : nullptr);
    float4* o = rec + 4 * (size_t)i;
    o[0] = make_float4(r[0], r[1], r[2], r[3]);
    o[1] = make_float4(r[4], r[5], r[6], r[7]);
    o[2] = make_float4(r[8], r[9], r[10], r[11]);
    o[3] = make_float4(r[12], r[13], r[14], r[15]);
    const uint32_t m = tm[i];
    if (m >= n_mat) atomicOr(err, 1u);
    aux[i] = Aux{0.0f, m, i, 0u};
}

// models: n_models x (M, inverse transpose) = 25 floats each, or null (world-space cones)
__global__ void k_flatten_cones(const float4* __restrict__ b, const float4* __restrict__ a,
                                const uint32_t* __restrict__ cm, const uint32_t* __restrict__ cmod,
                                const float* __restrict__ models, uint32_t n_models, uint32_t n_cones, uint32_t id0,
                                uint32_t n_mat, float4* rec, Aux* aux, float* bounds, float* cen, float* cone_h,
                                uint32_t* err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_cones) return;
    const uint32_t id = id0 + i;
    const float4 bb = b[i], aa = a[i];
    const v3 base = mk(bb.x, bb.y, bb.z), apex = mk(aa.x, aa.y, aa.z);
    float r[16];
    float base_d;
    if (models) {
        uint32_t k = cmod ? cmod[i] : 0u;
        if (k >= n_models) {
            atomicOr(err, 4u);
            k = 0;
        }
        const float* M = models + 25 * (size_t)k;
        base_d = cone_object_xf(base, apex, bb.w, aa.w, M, M + 16, r, bounds + 6 * (size_t)id, cen + 3 * (size_t)id);
    } else {
        base_d = cone_object(base, apex, bb.w, aa.w, r, bounds + 6 * (size_t)id, cen + 3 * (size_t)id);
    }
    if (cone_h) cone_h[i] = length(apex - base);  // Cylinder::m_height (pre-transform)
    float4* o = rec + 4 * (size_t)id;
    o[0] = make_float4(r[0], r[1], r[2], r[3]);
    o[1] = make_float4(r[4], r[5], r[6], r[7]);
    o[2] = make_float4(r[8], r[9], r[10], r[11]);
    o[3] = make_float4(r[12], r[13], r[14], r[15]);
    const uint32_t m = cm[i];
    if (m >= n_mat) atomicOr(err, 2u);
    aux[id] = Aux{base_d, m, id, 1u};
}

struct LnTable {
    float v[65];
};

// one strand per thread: positions / radii in private memory, then its
// verts-1 cones (khp_gen_hairball followed by khp_fibers_to_cones)
__global__ void k_gen_hairball(uint32_t n, uint32_t verts, float cx, float cy, float cz, float ball_r, float root_r,
                               uint32_t key0, LnTable lnt, float4* base_r0, float4* apex_r1) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    float P[3 * 64], R[64];
    hairball_strand(s, verts, mk(cx, cy, cz), ball_r, root_r, key0, lnt.v, P, R);
    const size_t k0 = (size_t)s * (verts - 1);
    for (uint32_t c = 0; c + 1 < verts; ++c) {
        float ob[4], oa[4];
        fiber_segment(P, R, c, ob, oa);
        base_r0[k0 + c] = make_float4(ob[0], ob[1], ob[2], ob[3]);
        apex_r1[k0 + c] = make_float4(oa[0], oa[1], oa[2], oa[3]);
    }
}

// one triangle per thread: strand s = t / (segs * per_seg) regenerated per
// thread (cheap next to the tube math), then fiber_tube_triangle
__global__ void k_gen_hairball_tris(uint32_t n, uint32_t verts, float cx, float cy, float cz, float ball_r,
                                    float root_r, uint32_t key0, LnTable lnt, uint32_t res, float* ov, float* on,
                                    float* of) {
    const uint32_t per_seg = 2 * res * res, per_strand = (verts - 1) * per_seg;
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)n * per_strand) return;
    const uint32_t s = (uint32_t)(t / per_strand), r = (uint32_t)(t % per_strand);
    float P[3 * 64], R[64];
    hairball_strand(s, verts, mk(cx, cy, cz), ball_r, root_r, key0, lnt.v, P, R);
    fiber_tube_triangle(P, R, r / per_seg, res, r % per_seg, ov + 9 * t, on + 9 * t, of + 9 * t);
}

#define FLCHK(expr)                                                                  \
    do {                                                                             \
        hipError_t e_ = (expr);                                                      \
        if (e_ != hipSuccess) return std::string(#expr) + ": " + hipGetErrorString(e_); \
    } while (0)

static uint32_t blocks(uint64_t n, uint32_t b) { return (uint32_t)((n + b - 1) / b); }

}  // namespace fl

std::string device_flatten(const khp_scene* s, bool device_ptrs, uint32_t n_materials, bool textured,
                           const std::vector<float>& models, DeviceObjects& o, hipStream_t st, double* kernel_ms) {
    using namespace fl;
    const uint32_t nt = s->n_tris, nc = s->n_cones, N = nt + nc;
    o.n_obj = N;
    o.n_tris = nt;
    o.n_cones = nc;
    FLCHK(o.rec.ensure(64 * (size_t)N));
    FLCHK(o.aux.ensure(sizeof(Aux) * (size_t)N));
    FLCHK(o.bounds.ensure(24 * (size_t)N));
    FLCHK(o.centroid.ensure(12 * (size_t)N));
    FLCHK(o.tri_nrm.ensure(36 * (size_t)std::max(nt, 1u)));
    FLCHK(o.tri_frame.ensure(36 * (size_t)std::max(nt, 1u)));
    if (s->tri_frame && nt)
        FLCHK(hipMemcpyAsync(o.tri_frame.p, s->tri_frame, 36 * (size_t)nt,
                             device_ptrs ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st));
    else
        FLCHK(hipMemsetAsync(o.tri_frame.p, 0, 36 * (size_t)std::max(nt, 1u), st));
    if (textured) {
        FLCHK(o.tri_uv.ensure(24 * (size_t)std::max(nt, 1u)));
        FLCHK(o.cone_h.ensure(4 * (size_t)std::max(nc, 1u)));
    } else {
        o.tri_uv.release();
        o.cone_h.release();
    }
    DevMem tv, tn, tm, tuv, cb, ca, cm, cmod, dmodels, err;
    const float *dtv = s->tri_v, *dtn = s->tri_n, *dcb = s->cone_base_r0, *dca = s->cone_apex_r1;
    const float* duv = textured ? s->tri_uv : nullptr;
    const uint32_t *dtm = s->tri_mat, *dcm = s->cone_mat, *dcmod = s->cone_model;
    if (!models.empty()) {
        FLCHK(dmodels.ensure(4 * models.size()));
        FLCHK(hipMemcpyAsync(dmodels.p, models.data(), 4 * models.size(), hipMemcpyHostToDevice, st));
    }
    if (!device_ptrs) {  // the library copies the caller's host arrays (khp_set_scene contract)
        if (nt) {
            FLCHK(tv.ensure(36 * (size_t)nt));
            FLCHK(tn.ensure(36 * (size_t)nt));
            FLCHK(tm.ensure(4 * (size_t)nt));
            FLCHK(hipMemcpyAsync(tv.p, s->tri_v, 36 * (size_t)nt, hipMemcpyHostToDevice, st));
            FLCHK(hipMemcpyAsync(tn.p, s->tri_n, 36 * (size_t)nt, hipMemcpyHostToDevice, st));
            FLCHK(hipMemcpyAsync(tm.p, s->tri_mat, 4 * (size_t)nt, hipMemcpyHostToDevice, st));
            dtv = tv.as<float>();
            dtn = tn.as<float>();
            dtm = tm.as<uint32_t>();
            if (duv) {
                FLCHK(tuv.ensure(24 * (size_t)nt));
                FLCHK(hipMemcpyAsync(tuv.p, s->tri_uv, 24 * (size_t)nt, hipMemcpyHostToDevice, st));
                duv = tuv.as<float>();
            }
        }
        if (nc) {
            FLCHK(cb.ensure(16 * (size_t)nc));
            FLCHK(ca.ensure(16 * (size_t)nc));
            FLCHK(cm.ensure(4 * (size_t)nc));
            FLCHK(hipMemcpyAsync(cb.p, s->cone_base_r0, 16 * (size_t)nc, hipMemcpyHostToDevice, st));
            FLCHK(hipMemcpyAsync(ca.p, s->cone_apex_r1, 16 * (size_t)nc, hipMemcpyHostToDevice, st));
            FLCHK(hipMemcpyAsync(cm.p, s->cone_mat, 4 * (size_t)nc, hipMemcpyHostToDevice, st));
            dcb = cb.as<float>();
            dca = ca.as<float>();
            dcm = cm.as<uint32_t>();
            if (s->cone_model) {
                FLCHK(cmod.ensure(4 * (size_t)nc));
                FLCHK(hipMemcpyAsync(cmod.p, s->cone_model, 4 * (size_t)nc, hipMemcpyHostToDevice, st));
                dcmod = cmod.as<uint32_t>();
            }
        }
    }
    FLCHK(err.ensure(4));
    FLCHK(hipMemsetAsync(err.p, 0, 4, st));
    hipEvent_t e0, e1;
    FLCHK(hipEventCreate(&e0));
    FLCHK(hipEventCreate(&e1));
    FLCHK(hipEventRecord(e0, st));
    if (nt)
        hipLaunchKernelGGL(k_flatten_tris, dim3(blocks(nt, 256)), dim3(256), 0, st, dtv, dtn, dtm, duv, nt,
                           n_materials, o.rec.as<float4>(), o.aux.as<Aux>(), o.bounds.as<float>(),
                           o.centroid.as<float>(), o.tri_nrm.as<float>(), textured ? o.tri_uv.as<float>() : nullptr,
                           err.as<uint32_t>());
    if (nc)
        hipLaunchKernelGGL(k_flatten_cones, dim3(blocks(nc, 256)), dim3(256), 0, st, (const float4*)dcb,
                           (const float4*)dca, dcm, models.empty() ? nullptr : dcmod,
                           models.empty() ? nullptr : dmodels.as<float>(), (uint32_t)(models.size() / 25), nc, nt,
                           n_materials, o.rec.as<float4>(), o.aux.as<Aux>(), o.bounds.as<float>(),
                           o.centroid.as<float>(), textured ? o.cone_h.as<float>() : nullptr, err.as<uint32_t>());
    FLCHK(hipGetLastError());
    FLCHK(hipEventRecord(e1, st));
    uint32_t herr = 0;
    FLCHK(hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, st));
    FLCHK(hipStreamSynchronize(st));
    float ms = 0.0f;
    FLCHK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (kernel_ms) *kernel_ms = ms;
    if (herr & 1u) return "EINVAL:triangle material index out of range";
    if (herr & 2u) return "EINVAL:cone material index out of range";
    if (herr & 4u) return "EINVAL:cone model index out of range";
    return std::string();
}

std::string device_gen_hairball(uint32_t n, uint32_t verts, const float center[3], float ball_r, float root_r,
                                uint32_t seed, float* d_base_r0, float* d_apex_r1, hipStream_t st) {
    using namespace fl;
    LnTable t{};
    for (int i = 1; i <= 64; ++i) t.v[i] = (float)std::log((double)i);  // as khp_gen_hairball
    const uint32_t key0 = lowbias32(seed ^ 0x48414952u);
    if (n)
        hipLaunchKernelGGL(k_gen_hairball, dim3(blocks(n, 128)), dim3(128), 0, st, n, verts, center[0], center[1],
                           center[2], ball_r, root_r, key0, t, (float4*)d_base_r0, (float4*)d_apex_r1);
    FLCHK(hipGetLastError());
    FLCHK(hipStreamSynchronize(st));
    return std::string();
}

std::string device_gen_hairball_tris(uint32_t n, uint32_t verts, const float center[3], float ball_r, float root_r,
                                     uint32_t seed, uint32_t res, float* d_v, float* d_n, float* d_frame,
                                     hipStream_t st) {
    using namespace fl;
    LnTable t{};
    for (int i = 1; i <= 64; ++i) t.v[i] = (float)std::log((double)i);
    const uint32_t key0 = lowbias32(seed ^ 0x48414952u);
    const size_t nt = (size_t)n * (verts - 1) * 2 * res * res;
    if (nt)
        hipLaunchKernelGGL(k_gen_hairball_tris, dim3((uint32_t)((nt + 127) / 128)), dim3(128), 0, st, n, verts,
                           center[0], center[1], center[2], ball_r, root_r, key0, t, res, d_v, d_n, d_frame);
    FLCHK(hipGetLastError());
    FLCHK(hipStreamSynchronize(st));
    return std::string();
}

}  // namespace khp

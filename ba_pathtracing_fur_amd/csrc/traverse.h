// traverse.h -- BVH2 traversal for KIRK's closest-hit and any-hit queries,
// written as a resumable per-lane step so persistent kernels can refill lanes.
//
// Semantics: BVH::closestIntersection / BVHNode::traverse(Intersection*) /
// Container::closestIntersectionWithCandidates (CPU_BVH.cpp:51-69, 148-199;
// Container.cpp:13-25) and their any-hit twins (CPU_BVH.cpp:77-93, 211-265;
// Container.cpp:27-34).  KIRK recurses near-child-first; an explicit stack of
// (ref, tmin, tmax) that pushes far-then-near and tests the prune condition at
// pop time visits exactly the same nodes in the same order, which matters
// because a leaf may accept a root beyond its own exit distance (SURVEY
// Appendix A.8/A.9) -- so the closest hit depends on the order.
//
// Stack policies: PrivStack (per-lane array; the batch query kernels) and
// LdsStack<R> (an R-entry ring per lane in LDS, striped [entry][lane] so a
// wave's accesses are bank-conflict free, spilling its oldest entries to a
// per-lane global area only when deeper than R).
#pragma once
// (included from device.h inside namespace khp)

struct Hit {
    float t;
    int32_t slot;
    float u, v;
};

struct TravStats {
    uint32_t nodes, prims;
};

struct TravRay {
    Ray r;
    v3 inv;
};

__device__ __forceinline__ void trav_setup(TravRay& tr, const Ray& r) {
    tr.r = r;
    tr.inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
}

__device__ __forceinline__ bool ref_leaf(uint32_t r) { return (r & LEAF_BIT) != 0u; }

struct PrivStack {
    uint32_t ref[STACK_MAX];
    float t0[STACK_MAX], t1[STACK_MAX];
    int sp;
    __device__ __forceinline__ void clear() { sp = 0; }
    __device__ __forceinline__ bool empty() const { return sp == 0; }
    __device__ __forceinline__ void push(uint32_t r, float a, float b) {
        ref[sp] = r;
        t0[sp] = a;
        t1[sp] = b;
        ++sp;
    }
    __device__ __forceinline__ void pop(uint32_t& r, float& a, float& b) {
        --sp;
        r = ref[sp];
        a = t0[sp];
        b = t1[sp];
    }
};

// The LDS image is three [R][256] arrays (ref, tmin bits, tmax bits) at the
// start of the kernel's dynamic LDS; a lane's column starts at its threadIdx.x.
// The spill area is [STACK_MAX][grid lanes] int4, addressed from blockIdx /
// threadIdx only on the (rare) spill path, so it costs no registers.
template <int R, bool COUNT>
struct LdsStack {
    static_assert((R & (R - 1)) == 0, "ring size must be a power of two");
    uint32_t* lds;
    int4* spill;
    uint32_t stride;
    int sp, lo;       // entries [0, lo) spilled to global, [lo, sp) in the LDS ring
    uint32_t spills;  // spill events (COUNT builds only)
    __device__ __forceinline__ void init(uint32_t* lds_base, int4* spill_base, uint32_t grid_lanes) {
        lds = lds_base;
        spill = spill_base;
        stride = grid_lanes;
        sp = lo = 0;
        spills = 0;
    }
    __device__ __forceinline__ void clear() { sp = lo = 0; }
    __device__ __forceinline__ bool empty() const { return sp == 0; }
    __device__ __forceinline__ uint32_t slot(int e) const { return (uint32_t)(e & (R - 1)) * 256u + threadIdx.x; }
    __device__ __forceinline__ int4* gcell(int e) const {
        return spill + (size_t)e * stride + blockIdx.x * blockDim.x + threadIdx.x;
    }
    __device__ __forceinline__ void push(uint32_t r, float a, float b) {
        if (sp - lo == R) {  // ring full: move the oldest entry to the spill column
            uint32_t k = slot(lo);
            *gcell(lo) = make_int4((int)lds[k], (int)lds[k + R * 256], (int)lds[k + 2 * R * 256], 0);
            ++lo;
            if (COUNT) ++spills;
        }
        uint32_t k = slot(sp);
        lds[k] = r;
        lds[k + R * 256] = bits_from_f(a);
        lds[k + 2 * R * 256] = bits_from_f(b);
        ++sp;
    }
    __device__ __forceinline__ void pop(uint32_t& r, float& a, float& b) {
        --sp;
        if (sp >= lo) {
            uint32_t k = slot(sp);
            r = lds[k];
            a = f_from_bits(lds[k + R * 256]);
            b = f_from_bits(lds[k + 2 * R * 256]);
        } else {
            int4 e = *gcell(sp);
            r = (uint32_t)e.x;
            a = f_from_bits((uint32_t)e.y);
            b = f_from_bits((uint32_t)e.z);
            lo = sp;
        }
    }
};

// Root box test (BVH::closestIntersection / isIntersection pre-test) and push.
template <class Stack>
__device__ __forceinline__ bool trav_begin(const DevScene& S, const TravRay& tr, Stack& stk) {
    stk.clear();
    float t0, t1;
    if (!slab(S.root_box[0], S.root_box[1], S.root_box[2], S.root_box[3], S.root_box[4], S.root_box[5], tr.r, tr.inv,
              t0, t1))
        return false;
    stk.push((uint32_t)S.root_ref, t0, t1);
    return true;
}

__device__ __forceinline__ uint32_t leaf_count(const DevScene& S, uint32_t ref) {
    uint32_t c = (ref >> 24) & 0x7Fu;
    if (c == LEAF_CNT_ESC) c = S.aux[ref & 0x00FFFFFFu].flags >> 8;
    return c;
}

// Push the children of an interior node in KIRK's order (near child popped first).
template <class Stack>
__device__ __forceinline__ void visit_interior(const DevScene& S, const TravRay& tr, uint32_t ref, Stack& stk) {
    const float4* np = reinterpret_cast<const float4*>(S.nodes + ref);
    float4 a = np[0], b = np[1], c = np[2];
    int4 rf = reinterpret_cast<const int4*>(np)[3];
    float l0, l1, r0, r1;
    bool lh = slab(a.x, a.y, a.z, a.w, b.x, b.y, tr.r, tr.inv, l0, l1);
    bool rh = slab(b.z, b.w, c.x, c.y, c.z, c.w, tr.r, tr.inv, r0, r1);
    if (lh && rh) {
        if (l0 < r0) {
            stk.push((uint32_t)rf.y, r0, r1);
            stk.push((uint32_t)rf.x, l0, l1);
        } else {
            stk.push((uint32_t)rf.x, l0, l1);
            stk.push((uint32_t)rf.y, r0, r1);
        }
    } else if (lh) {
        stk.push((uint32_t)rf.x, l0, l1);
    } else if (rh) {
        stk.push((uint32_t)rf.y, r0, r1);
    }
}

// One closest-hit step: pop one entry and process it.
template <bool STATS, class Stack>
__device__ __forceinline__ void closest_step(const DevScene& S, const TravRay& tr, Hit& h, Stack& stk,
                                             TravStats& st) {
    uint32_t ref;
    float tmin, tmax;
    stk.pop(ref, tmin, tmax);
    if (tmax < 0.0f || tmin > h.t) return;
    if (STATS) st.nodes++;
    if (ref_leaf(ref)) {
        const uint32_t first = ref & 0x00FFFFFFu, cnt = leaf_count(S, ref);
        float tl = FLT_MAX_, lu = 0.0f, lv = 0.0f, tMax = tmax;
        int32_t sl = -1;
        for (uint32_t k = 0; k < cnt; ++k) {
            const int32_t slot = (int32_t)(first + k);
            const float4* p = S.prims + 4 * (size_t)slot;
            float4 p0 = p[0], p1 = p[1], p2 = p[2];
            if (STATS) st.prims++;
            float t, u = 0.0f, v = 0.0f;
            bool ok;
            if (is_tri(p0)) ok = tri_test(p0, p1, p2, tr.r, 0.0f, tMax, t, u, v);
            else ok = cone_closest(p0, p1, p2, p[3], tr.r, 0.0f, tMax, t);
            if (ok) {
                tl = t;
                sl = slot;
                lu = u;
                lv = v;
                tMax = t;
            }
        }
        if (sl >= 0 && tl < h.t) {
            h.t = tl;
            h.slot = sl;
            h.u = lu;
            h.v = lv;
        }
    } else {
        visit_interior(S, tr, ref, stk);
    }
}

// One any-hit step; returns true when an occluder is found.
template <bool STATS, class Stack>
__device__ __forceinline__ bool any_step(const DevScene& S, const TravRay& tr, float tMaxRay, Stack& stk,
                                         TravStats& st) {
    uint32_t ref;
    float tmin, tmax;
    stk.pop(ref, tmin, tmax);
    if (tmax < 0.0f || tmin > tMaxRay) return false;
    if (STATS) st.nodes++;
    if (ref_leaf(ref)) {
        const uint32_t first = ref & 0x00FFFFFFu, cnt = leaf_count(S, ref);
        for (uint32_t k = 0; k < cnt; ++k) {
            const float4* p = S.prims + 4 * (size_t)(first + k);
            float4 p0 = p[0], p1 = p[1], p2 = p[2];
            if (STATS) st.prims++;
            bool ok;
            if (is_tri(p0)) {
                float t, u, v;
                ok = tri_test(p0, p1, p2, tr.r, 0.0f, tMaxRay, t, u, v);
            } else {
                ok = cone_any(p0, p1, p2, p[3], tr.r, tMaxRay);
            }
            if (ok) return true;
        }
        return false;
    }
    visit_interior(S, tr, ref, stk);
    return false;
}

// Whole-ray forms (batch query kernels).
template <bool STATS, class Stack>
__device__ __forceinline__ void trace_closest(const DevScene& S, const Ray& r, Hit& h, Stack& stk, TravStats& st) {
    h.t = FLT_MAX_;
    h.slot = -1;
    h.u = h.v = 0.0f;
    TravRay tr;
    trav_setup(tr, r);
    if (!trav_begin(S, tr, stk)) return;
    while (!stk.empty()) closest_step<STATS>(S, tr, h, stk, st);
}

template <bool STATS, class Stack>
__device__ __forceinline__ bool trace_any(const DevScene& S, const Ray& r, float tMaxRay, Stack& stk, TravStats& st) {
    TravRay tr;
    trav_setup(tr, r);
    if (!trav_begin(S, tr, stk)) return false;
    while (!stk.empty())
        if (any_step<STATS>(S, tr, tMaxRay, stk, st)) return true;
    return false;
}

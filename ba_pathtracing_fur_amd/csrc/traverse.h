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
    uint32_t nodes, prims, pruned;  // pruned: entries popped only to fail the prune test
};

struct TravRay {
    Ray r;
    v3 inv;
    bool fin;  // origin and inverse direction finite on every axis (the fast slab test is exact)
};

__device__ __forceinline__ void trav_setup(TravRay& tr, const Ray& r) {
    tr.r = r;
    tr.inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    tr.fin = __builtin_isfinite(tr.inv.x) && __builtin_isfinite(tr.inv.y) && __builtin_isfinite(tr.inv.z) &&
             __builtin_isfinite(r.o.x) && __builtin_isfinite(r.o.y) && __builtin_isfinite(r.o.z);
}

// NaN rays (a BSDF can return a NaN direction, e.g. at KIRK's grazing-angle
// divisions; KIRK traces them like any other ray, CPU_PathTracer.cpp:172).
// Their results follow from IEEE comparisons alone, without the traversal:
//  * closest hit: every cone test fails (its quadratic is NaN, so no
//    accept comparison holds) and every triangle test that passes returns
//    t = NaN, which never satisfies the leaf's `tl < hit.t` -- so a ray with
//    a NaN in its origin or direction ends with no hit;
//  * any hit, NaN x direction (inv.x NaN): every slab returns true with
//    t0 = t1 = NaN (the x entry/exit stay NaN, no later comparison replaces or
//    rejects them), nothing is pruned, cones fail, and every triangle passes
//    (det NaN -> u, v, t NaN, no rejecting comparison holds) -- so the ray is
//    occluded iff the scene has a triangle.
// KIRK walks the whole BVH for such a ray (about 20M records at config 5:
// seconds per launch).  The instrumented kernels keep the walk, so KIRK's
// visit counts stay exact there.
__device__ __forceinline__ bool ray_has_nan(const Ray& r) {
    return r.o.x != r.o.x || r.o.y != r.o.y || r.o.z != r.o.z || r.d.x != r.d.x || r.d.y != r.d.y ||
           r.d.z != r.d.z;
}

// Any hit for rays whose x slab is NaN: a NaN origin x or a NaN inverse
// direction x (shadow rays from a hit whose normal is NaN get a NaN origin and
// a finite direction).  The x entry/exit of every box is then NaN and stays
// NaN through BoundingVolume::intersects' comparisons, so every box passes
// and nothing is pruned: KIRK visits every node and tests every candidate
// until one passes.  Cones never pass (their quadratic is NaN).  A triangle
// passes iff its determinant passes the |det| < eps rejection: u, v and t
// are NaN (NaN origin) and no rejecting comparison holds; with a NaN direction
// the determinant itself is NaN.  The answer does not depend on the visit
// order, so it is "some triangle has !(|det| < eps)", found here in object
// order (usually at the first triangle) instead of KIRK's walk of the whole
// tree, which took ~10 s for one such ray at config 3.
__device__ __forceinline__ bool x_slab_nan(const TravRay& tr) { return tr.inv.x != tr.inv.x || tr.r.o.x != tr.r.o.x; }
__device__ __forceinline__ bool any_hit_x_nan(const DevScene& S, const Ray& r) {
    for (uint32_t k = 0; k < S.n_tris; ++k) {
        const float4* p = S.prims + 4 * (size_t)S.tri_slot[k];
        const float4 ab = p[1], ac = p[2];  // tri_test's det: dot(cross(d, ac), ab)
        const v3 dv = cross(r.d, mk(ac.x, ac.y, ac.z));
        const float det = dot(dv, mk(ab.x, ab.y, ab.z));
        if (!(fabsf(det) < TRI_EPS_D)) return true;
    }
    return false;
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

// Threads per block of the persistent traversal kernels.  One wave per block:
// a block's LDS is released only when all of its waves have ended, so with
// 4-wave blocks a launch's tail (a few long rays scattered over many blocks)
// kept most of the chip's LDS allocated and no other kernel could start
// there; with 1-wave blocks each finished wave frees its share at once.
#ifndef KHP_TRAV_BLOCK
#define KHP_TRAV_BLOCK 64
#endif
constexpr uint32_t TRAV_BLOCK = KHP_TRAV_BLOCK;

// The LDS image is three [R][TRAV_BLOCK] arrays (ref, tmin bits, tmax bits) at the
// start of the kernel's dynamic LDS; a lane's column starts at its threadIdx.x.
// The spill area is [STACK_MAX][grid lanes] int4, addressed from blockIdx /
// threadIdx only on the (rare) spill path, so it costs no registers.
// Top-of-tree staging (khp_ctx_params.lds_nodes, SURVEY north_star "node records
// staged in LDS"): a kernel instance with TOP stages the tree's top TOP_NODES
// interior records (three levels) after its rings, and a ref with TOP_REF set
// (interior refs keep bits 24-30 clear) names one of them.
constexpr uint32_t TOP_NODES = 7;
constexpr uint32_t TOP_REF = 0x40000000u;
template <int R, bool COUNT, bool TOP = false>
struct LdsStack {
    static_assert(R >= 2 && R <= 16, "ring size");
    static constexpr bool kTop = TOP;
    static constexpr size_t kRingBytes = 3 * (size_t)R * TRAV_BLOCK * sizeof(uint32_t);
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
    // the staged top records (TOP instances; read-only after stage_top)
    __device__ __forceinline__ const float4* top() const {
        return reinterpret_cast<const float4*>(lds + 3 * R * TRAV_BLOCK);
    }
    // Copies the top records into this block's LDS (one-wave blocks: every lane
    // takes part, then a barrier).
    __device__ __forceinline__ void stage_top(const float4* __restrict__ src) {
        float4* dst = reinterpret_cast<float4*>(lds + 3 * R * TRAV_BLOCK);
        for (uint32_t i = threadIdx.x; i < 4 * TOP_NODES; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
    __device__ __forceinline__ void clear() { sp = lo = 0; }
    __device__ __forceinline__ bool empty() const { return sp == 0; }
    __device__ __forceinline__ uint32_t slot(int e) const { return (uint32_t)((uint32_t)e % (uint32_t)R) * TRAV_BLOCK + threadIdx.x; }
    __device__ __forceinline__ int4* gcell(int e) const {
        return spill + (size_t)e * stride + blockIdx.x * blockDim.x + threadIdx.x;
    }
    __device__ __forceinline__ void push(uint32_t r, float a, float b) {
        if (sp - lo == R) {  // ring full: move the oldest entry to the spill column
            uint32_t k = slot(lo);
            *gcell(lo) = make_int4((int)lds[k], (int)lds[k + R * TRAV_BLOCK], (int)lds[k + 2 * R * TRAV_BLOCK], 0);
            ++lo;
            if (COUNT) ++spills;
        }
        uint32_t k = slot(sp);
        lds[k] = r;
        lds[k + R * TRAV_BLOCK] = bits_from_f(a);
        lds[k + 2 * R * TRAV_BLOCK] = bits_from_f(b);
        ++sp;
    }
    // The ring slot is read unconditionally (a stale but harmless slot when
    // the entry was spilled), pinned, and the rare spill read overrides it.
    // Otherwise the compiler merges both reads into FLAT loads through a
    // selected pointer: 3 extra vector-memory instructions and a vmcnt(0)
    // wait on every pop.
    __device__ __forceinline__ void pop(uint32_t& r, float& a, float& b) {
        --sp;
        const uint32_t k = slot(sp);
        r = lds[k];
        a = f_from_bits(lds[k + R * TRAV_BLOCK]);
        b = f_from_bits(lds[k + 2 * R * TRAV_BLOCK]);
        asm volatile("" : "+v"(r), "+v"(a), "+v"(b));  // the LDS reads happen here
        if (sp < lo) {
            int4 e = *gcell(sp);
            r = (uint32_t)e.x;
            a = f_from_bits((uint32_t)e.y);
            b = f_from_bits((uint32_t)e.z);
            lo = sp;
        }
    }
};

// Materialise a fetched record in registers at this point.  Without it the
// compiler splits a 64-B record fetch and sinks the loads of the fields a test
// needs late (z planes, the cone's W / max_d) below the test's early-out
// branches, which turns one memory round trip per record into two or three
// dependent ones (seen in the gfx950 ISA).
__device__ __forceinline__ void pin(float4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
__device__ __forceinline__ void pin(int4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }

// The entry a lane processes next lives in registers (Cur); the stack holds
// only the deferred far children.  When both children of a node are hit,
// KIRK's recursion descends into the nearer one first: here it becomes `cur`
// directly and the farther one is pushed -- the same visit order as
// push(far), push(near), pop() without the LDS round trip.
struct Cur {
    uint32_t ref;
    float t0, t1;
    bool valid;
};

template <class Stack>
__device__ __forceinline__ void cur_next(Stack& stk, Cur& c) {
    if (stk.empty()) {
        c.valid = false;
    } else {
        stk.pop(c.ref, c.t0, c.t1);
        c.valid = true;
    }
}


// Root box test (BVH::closestIntersection / isIntersection pre-test).
template <class Stack>
__device__ __forceinline__ bool trav_begin(const DevScene& S, const TravRay& tr, Stack& stk, Cur& c) {
    stk.clear();
    float t0, t1;
    c.valid = slab(S.root_box[0], S.root_box[1], S.root_box[2], S.root_box[3], S.root_box[4], S.root_box[5], tr.r,
                   tr.inv, t0, t1);
    c.ref = (uint32_t)S.root_ref;
    c.t0 = t0;
    c.t1 = t1;
    return c.valid;
}

__device__ __forceinline__ uint32_t leaf_count(const DevScene& S, uint32_t ref) {
    uint32_t c = (ref >> 24) & 0x7Fu;
    if (c == LEAF_CNT_ESC) c = S.aux[ref & 0x00FFFFFFu].flags >> 8;
    return c;
}

// Interior entry: prune test (BVHNode::traverse, CPU_BVH.cpp:151-153) at the
// moment KIRK would pop it, then both child boxes, near child first.
// tlimit = current closest t (closest hit) or the ray's tMax (any hit).
template <bool STATS, class Stack>
__device__ __forceinline__ void interior_step(const DevScene& S, const TravRay& tr, float tlimit, Stack& stk, Cur& c,
                                              TravStats& st) {
    if (c.t1 < 0.0f || c.t0 > tlimit) {
        cur_next(stk, c);
        return;
    }
    if (STATS) st.nodes++;
    const float4* np = reinterpret_cast<const float4*>(S.nodes + c.ref);
    float4 a = np[0], b = np[1], cc = np[2];
    int4 rf = reinterpret_cast<const int4*>(np)[3];
    pin(a);
    pin(b);
    pin(cc);
    pin(rf);
    float l0, l1, r0, r1;
    bool lh = slab(a.x, a.y, a.z, a.w, b.x, b.y, tr.r, tr.inv, l0, l1);
    bool rh = slab(b.z, b.w, cc.x, cc.y, cc.z, cc.w, tr.r, tr.inv, r0, r1);
    if (lh && rh) {
        if (l0 < r0) {
            stk.push((uint32_t)rf.y, r0, r1);
            c = Cur{(uint32_t)rf.x, l0, l1, true};
        } else {
            stk.push((uint32_t)rf.x, l0, l1);
            c = Cur{(uint32_t)rf.y, r0, r1, true};
        }
    } else if (lh) {
        c = Cur{(uint32_t)rf.x, l0, l1, true};
    } else if (rh) {
        c = Cur{(uint32_t)rf.y, r0, r1, true};
    } else {
        cur_next(stk, c);
    }
}

// One candidate of a leaf (Container::closestIntersectionWithCandidates,
// Container.cpp:13-25): window [0, tMax], later equal-t candidates overwrite.
__device__ __forceinline__ void leaf_candidate(float4 p0, float4 p1, float4 p2, float4 p3, int32_t slot,
                                               const Ray& r, float& tMax, float& tl, int32_t& sl, float& lu,
                                               float& lv) {
    float t, u = 0.0f, v = 0.0f;
    bool ok;
    if (is_tri(p0)) ok = tri_test(p0, p1, p2, r, 0.0f, tMax, t, u, v);
    else ok = cone_closest(p0, p1, p2, p3, r, 0.0f, tMax, t);
    if (ok) {
        tl = t;
        sl = slot;
        lu = u;
        lv = v;
        tMax = t;
    }
}

// Leaf entry, closest hit: prune test, then every candidate with tMin = 0 and
// tMax = the leaf's exit distance (CPU_BVH.cpp:155-167).
template <bool STATS, class Stack>
__device__ __forceinline__ void leaf_step_closest(const DevScene& S, const TravRay& tr, Hit& h, Stack& stk, Cur& c,
                                                  TravStats& st) {
    if (!(c.t1 < 0.0f || c.t0 > h.t)) {
        if (STATS) st.nodes++;
        const uint32_t first = c.ref & 0x00FFFFFFu, cnt = leaf_count(S, c.ref);
        const float4* p = S.prims + 4 * (size_t)first;
        float tl = FLT_MAX_, lu = 0.0f, lv = 0.0f, tMax = c.t1;
        int32_t sl = -1;
        if (STATS) st.prims += cnt;
        for (uint32_t k = 0; k < cnt; ++k) {
            const float4* q = p + 4 * k;
            float4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
            pin(q0);
            pin(q1);
            pin(q2);
            pin(q3);
            leaf_candidate(q0, q1, q2, q3, (int32_t)(first + k), tr.r, tMax, tl, sl, lu, lv);
        }
        if (sl >= 0 && tl < h.t) {
            h.t = tl;
            h.slot = sl;
            h.u = lu;
            h.v = lv;
        }
    }
    cur_next(stk, c);
}

// leaf_candidate without the barycentrics (the production closest-hit loops):
// the leaf's best t is its shrunk window tMax whenever a candidate was
// accepted (sl >= 0), and u, v are recomputed from the hit (tri_uv).
__device__ __forceinline__ void leaf_candidate_t(float4 p0, float4 p1, float4 p2, float4 p3, int32_t slot,
                                                 const Ray& r, float& tMax, int32_t& sl) {
    float t, u, v;
    bool ok;
    if (is_tri(p0)) ok = tri_test(p0, p1, p2, r, 0.0f, tMax, t, u, v);
    else ok = cone_closest(p0, p1, p2, p3, r, 0.0f, tMax, t);
    if (ok) {
        sl = slot;
        tMax = t;
    }
}

__device__ __forceinline__ bool any_candidate(float4 p0, float4 p1, float4 p2, float4 p3, const Ray& r,
                                              float tMaxRay) {
    if (is_tri(p0)) {
        float t, u, v;
        return tri_test(p0, p1, p2, r, 0.0f, tMaxRay, t, u, v);
    }
    return cone_any(p0, p1, p2, p3, r, tMaxRay);
}

// Leaf entry, any hit (BVHNode::traverse(ray), CPU_BVH.cpp:211-265; Container.cpp:27-34).
// Returns true when an occluder is found (traversal ends).
template <bool STATS, class Stack>
__device__ __forceinline__ bool leaf_step_any(const DevScene& S, const TravRay& tr, float tMaxRay, Stack& stk, Cur& c,
                                              TravStats& st) {
    if (!(c.t1 < 0.0f || c.t0 > tMaxRay)) {
        if (STATS) st.nodes++;
        const uint32_t first = c.ref & 0x00FFFFFFu, cnt = leaf_count(S, c.ref);
        const float4* p = S.prims + 4 * (size_t)first;
        for (uint32_t k = 0; k < cnt; ++k) {
            const float4* q = p + 4 * k;
            float4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3];
            pin(q0);
            pin(q1);
            pin(q2);
            pin(q3);
            if (STATS) st.prims++;
            if (any_candidate(q0, q1, q2, q3, tr.r, tMaxRay)) return true;
        }
    }
    cur_next(stk, c);
    return false;
}

// ---- select-based one-fetch loop (the production kernels) -------------------------------
// A lane holds either an interior entry (cursor) or a partly tested leaf
// (LeafCur).  Each wave iteration loads exactly ONE 64-B record -- a node or
// a candidate primitive -- through one instruction stream, runs the slab pair
// or the one candidate test, and does at most one push and one pop, with every
// branch written as selects.  The divergent form this replaced (a pop inside
// every branch and a pop loop) cost ~185 SALU instructions per wave iteration
// on exec-mask bookkeeping; the scalar unit, which the 4 SIMDs of a CU share,
// was ~75 % busy (profiles/r01g, `mix` pass).
// A lane is in one of four modes:
//   M_NODE  the cursor (c) is an interior entry that passed its prune test;
//   M_LEAF  the lane is testing the candidates of an opened leaf (lf);
//   M_POP   the lane must pop its next entry (set when a popped entry failed
//           its prune test: instead of looping, the lane pops again in the
//           next iteration -- 1.2 such pops per ray against ~110 iterations);
//   M_IDLE  no ray.
// Visit order and arithmetic are those of interior_step / leaf_step_*:
// candidates of a leaf are tested in order with the leaf's window, and entries
// are prune-tested exactly when KIRK would pop them.  Push-time pruning: a
// child that would fail the prune test `t1 < 0 || t0 > tlimit` when popped is
// dropped at once -- tlimit only ever decreases (closest hit) or is fixed (any
// hit), so it is certain to be pruned later; the live entries, their order and
// every visit (the counts included) are unchanged.
struct LeafCur {
    uint32_t slot, left;  // next candidate slot, candidates still to test (0: not in a leaf)
    float tmax;           // closest: the leaf window (shrinks on hits); any: unused
    float tl, lu, lv;     // closest: best candidate of this leaf so far
    int32_t sl;
};

enum : uint32_t { M_IDLE = 0u, M_NODE = 1u, M_LEAF = 2u, M_POP = 3u };

// BoundingVolume::intersects as selects: every IEEE operation of slab() is
// evaluated, the early-out tests are and-ed; t0/t1 are those of slab()
// whenever the result is true.
__device__ __forceinline__ bool slab_sel(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                         const TravRay& tr, float& t0, float& t1) {
    const bool sx = tr.r.d.x < 0.0f, sy = tr.r.d.y < 0.0f, sz = tr.r.d.z < 0.0f;
    float tmin = ((sx ? mxx : mnx) - tr.r.o.x) * tr.inv.x;
    float tmax = ((sx ? mnx : mxx) - tr.r.o.x) * tr.inv.x;
    const float tymin = ((sy ? mxy : mny) - tr.r.o.y) * tr.inv.y;
    const float tymax = ((sy ? mny : mxy) - tr.r.o.y) * tr.inv.y;
    bool ok = !((tmin > tymax) || (tymin > tmax));
    tmin = (tymin > tmin) ? tymin : tmin;
    tmax = (tymax < tmax) ? tymax : tmax;
    const float tzmin = ((sz ? mxz : mnz) - tr.r.o.z) * tr.inv.z;
    const float tzmax = ((sz ? mnz : mxz) - tr.r.o.z) * tr.inv.z;
    ok = ok && !((tmin > tzmax) || (tzmin > tmax));
    t0 = (tzmin > tmin) ? tzmin : tmin;
    t1 = (tzmax < tmax) ? tzmax : tmax;
    return ok;
}

// Fast slab pair for rays whose inverse direction is finite on every axis
// (every ray but those with an exactly zero direction component).  Then
// (mn - o)*inv and (mx - o)*inv are finite and ordered by the sign of inv, so
// min/max pick exactly the operands KIRK's sign selects pick, and KIRK's
// chain of early-out comparisons is equivalent to max3(entries) <= min3(exits)
// (each axis' own entry <= exit).  t0/t1 are bit-identical up to the sign of a
// zero, which no comparison downstream distinguishes.  Rays with an infinite
// component (0 * inf = NaN cases) take slab_sel.
__device__ __forceinline__ bool slab_fast(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                          const TravRay& tr, float& t0, float& t1) {
    const float ax = (mnx - tr.r.o.x) * tr.inv.x, bx = (mxx - tr.r.o.x) * tr.inv.x;
    const float ay = (mny - tr.r.o.y) * tr.inv.y, by = (mxy - tr.r.o.y) * tr.inv.y;
    const float az = (mnz - tr.r.o.z) * tr.inv.z, bz = (mxz - tr.r.o.z) * tr.inv.z;
    t0 = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    t1 = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz));
    return t0 <= t1;
}

// A new entry that passed its prune test becomes the lane's work: an interior
// node is fetched next iteration, a leaf is opened (KIRK's leaf prologue,
// CPU_BVH.cpp:155-159).
template <bool STATS>
__device__ __forceinline__ void take_entry(const DevScene& S, uint32_t ref, float t0, float t1, uint32_t& mode, Cur& c,
                                           LeafCur& lf, TravStats& st) {
    const bool leaf = ref_leaf(ref);
    c.ref = ref;
    c.t0 = t0;
    c.t1 = t1;
    mode = leaf ? M_LEAF : M_NODE;
    uint32_t cnt = (ref >> 24) & 0x7Fu;
    if (leaf && cnt == LEAF_CNT_ESC) cnt = S.aux[ref & 0x00FFFFFFu].flags >> 8;
    lf.slot = leaf ? (ref & 0x00FFFFFFu) : lf.slot;
    lf.left = leaf ? cnt : 0u;
    lf.tmax = t1;
    lf.tl = FLT_MAX_;
    lf.lu = 0.0f;
    lf.lv = 0.0f;
    lf.sl = -1;
    if (STATS && leaf) st.nodes++;
}

// Start a ray: root box pre-test (BVH::closestIntersection / isIntersection).
// Returns false when the ray misses the root box (finished at once).
template <bool STATS, class Stack>
__device__ __forceinline__ bool trav2_begin(const DevScene& S, const TravRay& tr, float tlimit, Stack& stk,
                                            uint32_t& mode, Cur& c, LeafCur& lf, TravStats& st) {
    stk.clear();
    float t0, t1;
    if (!slab(S.root_box[0], S.root_box[1], S.root_box[2], S.root_box[3], S.root_box[4], S.root_box[5], tr.r,
              tr.inv, t0, t1))
        return false;
    if (t1 < 0.0f || t0 > tlimit) {  // pruned at pop time: the next pop finds the stack empty
        if (STATS) st.pruned++;
        mode = M_POP;
        return true;
    }
    take_entry<STATS>(S, (uint32_t)(Stack::kTop ? S.top_root : S.root_ref), t0, t1, mode, c, lf, st);
    return true;
}

// A candidate of a leaf for a lane whose query kind is a per-lane value (the
// path kernel traces closest-hit and any-hit rays in one loop): the same test
// as leaf_candidate_t (any = false, window tMax = the leaf's) or any_candidate
// (any = true, tMax = the ray's), with one instruction stream for both.
__device__ __forceinline__ bool candidate_rt(float4 p0, float4 p1, float4 p2, float4 p3, const Ray& r, bool any,
                                             float tMax, float& t) {
    if (is_tri(p0)) {
        float u, v;
        return tri_test(p0, p1, p2, r, 0.0f, tMax, t, u, v);
    }
    return cone_quadratic(p0, p1, p2, p3, r, any, 0.0f, tMax, t);
}

#ifdef KHP_LEAF_REUSE
// Diagnostic builds: how many lanes of a wave fetch the SAME
// candidate (cone / triangle) record in one traversal iteration of the instrumented
// closest-hit kernels.  Per bounce (g_reuse_b, set by the host before each launch),
// the leaf-record fetches are binned by the size of their group of lanes fetching the
// same record: 1, 2, 3-4, 5-8, 9-16, 17-32, 33-64 (weighted by lanes), and slot 7
// counts the distinct records fetched.  Read by khp_debug_leaf_reuse.
__device__ unsigned long long g_leaf_hist[16 * 8];
__device__ uint32_t g_reuse_b;
__device__ __forceinline__ void leaf_reuse(bool in_leaf, uint32_t slot) {
    unsigned long long m = __ballot(in_leaf);
    const uint32_t b = g_reuse_b < 16u ? g_reuse_b : 15u;
    const uint32_t lane = threadIdx.x & 63u;
    while (m) {
        const int leader = __ffsll((long long)m) - 1;
        const uint32_t s = (uint32_t)__shfl((int)slot, leader);
        const unsigned long long same = __ballot(in_leaf && slot == s) & m;
        const uint32_t n = (uint32_t)__popcll(same);
        const uint32_t k = n == 1u ? 0u : n == 2u ? 1u : n <= 4u ? 2u : n <= 8u ? 3u : n <= 16u ? 4u : n <= 32u ? 5u : 6u;
        if (lane == (uint32_t)leader) {
            atomicAdd(&g_leaf_hist[b * 8 + k], (unsigned long long)n);
            atomicAdd(&g_leaf_hist[b * 8 + 7], 1ull);
        }
        m &= ~same;
    }
}
#endif

// One wave iteration of one lane (mode != M_IDLE).  KIND 1: any-hit with the
// fixed limit tlimit = the ray's tMax; KIND 0: closest hit, tlimit = h.t;
// KIND 2: the lane's any_rt decides (the path kernel).  Returns true when the
// ray is finished; for an any-hit query, `occluded` tells the result.
template <int KIND, bool STATS, class Stack>
__device__ __forceinline__ bool iter2k(const DevScene& S, const TravRay& tr, Hit& h, float tmax_any, Stack& stk,
                                       uint32_t& mode, Cur& c, LeafCur& lf, TravStats& st, bool& occluded,
                                       bool any_rt) {
    const bool ANY = KIND == 2 ? any_rt : KIND == 1;
    const bool in_leaf = mode == M_LEAF;
    const bool fetch = in_leaf || mode == M_NODE;
    const float4* p = in_leaf ? S.prims + 4 * (size_t)lf.slot : reinterpret_cast<const float4*>(S.nodes + c.ref);
#ifdef KHP_LEAF_REUSE
    if (STATS && KIND == 0) leaf_reuse(in_leaf, lf.slot);
#endif
    float4 q0, q1, q2, q3;
    if (Stack::kTop && fetch && !in_leaf && (c.ref & TOP_REF) != 0u) {   // a staged top record (LDS)
        const float4* t = stk.top() + 4 * (c.ref & 0xFFu);
        q0 = t[0];
        q1 = t[1];
        q2 = t[2];
        q3 = t[3];
    } else if (fetch) {
        q0 = p[0];
        q1 = p[1];
        q2 = p[2];
        q3 = p[3];
        pin(q0); pin(q1); pin(q2); pin(q3);
    }
    bool need_pop = mode == M_POP;
    bool have = false;  // a new entry (ref, t0, t1) for take_entry
    uint32_t eref = 0u;
    float et0 = 0.0f, et1 = 0.0f;
    bool push = false;
    uint32_t pref = 0u;
    float pt0 = 0.0f, pt1 = 0.0f;
    if (in_leaf) {
        if (STATS) st.prims++;
        if (KIND == 2) {
            float t = 0.0f;
            const bool ok = candidate_rt(q0, q1, q2, q3, tr.r, ANY, ANY ? tmax_any : lf.tmax, t);
            if (ok && ANY) {
                occluded = true;
                return true;
            }
            if (ok) {
                lf.sl = (int32_t)lf.slot;
                lf.tmax = t;
            }
        } else if (ANY) {
            if (any_candidate(q0, q1, q2, q3, tr.r, tmax_any)) {
                occluded = true;
                return true;
            }
        } else {
            leaf_candidate_t(q0, q1, q2, q3, (int32_t)lf.slot, tr.r, lf.tmax, lf.sl);
        }
        ++lf.slot;
        --lf.left;
        if (lf.left == 0u) {
            if (!ANY && lf.sl >= 0 && lf.tmax < h.t) {  // the leaf's best t is its window (leaf_candidate_t)
                h.t = lf.tmax;
                h.slot = lf.sl;
            }
            need_pop = true;
        }
    } else if (fetch) {
        if (STATS) st.nodes++;
        const float tlimit = ANY ? tmax_any : h.t;
        float l0, l1, r0, r1;
        bool lh, rh;
        if (__ballot(!tr.fin) == 0ull) {  // wave-uniform
            lh = slab_fast(q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, tr, l0, l1);
            rh = slab_fast(q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, tr, r0, r1);
        } else {
            lh = slab_sel(q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, tr, l0, l1);
            rh = slab_sel(q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, tr, r0, r1);
        }
        lh = lh && !(l1 < 0.0f || l0 > tlimit);
        rh = rh && !(r1 < 0.0f || r0 > tlimit);
        const uint32_t lref = __float_as_uint(q3.x), rref = __float_as_uint(q3.y);
        const bool nearl = lh && (!rh || l0 < r0);  // KIRK: left first iff l0 < r0 (ties: right)
        have = lh || rh;
        need_pop = !have;
        push = lh && rh;
        eref = nearl ? lref : rref;
        et0 = nearl ? l0 : r0;
        et1 = nearl ? l1 : r1;
        pref = nearl ? rref : lref;
        pt0 = nearl ? r0 : l0;
        pt1 = nearl ? r1 : l1;
    }
    if (push) stk.push(pref, pt0, pt1);
    if (need_pop) {
        if (stk.empty()) {
            mode = M_IDLE;
            occluded = false;
            return true;
        }
        stk.pop(eref, et0, et1);
        const float tlimit = ANY ? tmax_any : h.t;
        if (et1 < 0.0f || et0 > tlimit) {
            if (STATS) st.pruned++;
            mode = M_POP;
        } else {
            have = true;
        }
    }
    if (have) take_entry<STATS>(S, eref, et0, et1, mode, c, lf, st);
    return false;
}

template <bool ANY, bool STATS, class Stack>
__device__ __forceinline__ bool iter2(const DevScene& S, const TravRay& tr, Hit& h, float tmax_any, Stack& stk,
                                      uint32_t& mode, Cur& c, LeafCur& lf, TravStats& st, bool& occluded) {
    return iter2k<ANY ? 1 : 0, STATS>(S, tr, h, tmax_any, stk, mode, c, lf, st, occluded, ANY);
}

// ---- two-level node records (k_extend from bounce wide_from; k_shadow from bounce 2) -------
// The wide record of interior node X (one 128-B line, `DevScene::wide`, same
// index as X's 64-B record) holds, for each child C of X, either the boxes and
// refs of C's two children (C interior) or C's own box (C a leaf):
//   [0..2]  g0, g1 boxes   (child 1's children, or child 1's box in g0)
//   [3..5]  g2, g3 boxes   (the same for child 2)
//   [6]     ref c1, ref c2, ref g0, ref g1      [7] ref g2, ref g3, 0, 0
// Box k is (mn.xyz, mx.xyz) packed like DevNode's left/right pair.  C's own
// box is not stored: KIRK's node box is the union (std::min / std::max) of its
// objects' bounds (CPU_BVH.cpp:113-118), so it equals the union of its two
// children's boxes bit for bit -- checked for every node when the records are
// built (k_wide_records); a scene where it fails keeps the 64-B loop.  For a ray
// with finite origin and inverse direction, every per-axis plane distance
// (b - o) * inv is monotone in b, so C's per-axis entry / exit are exactly the
// min / max of its children's (both boxes ordered, mn <= mx, also checked), and
// slab_fast on C's box follows without C's bounds.
//
// One fetch then does the work of two of KIRK's levels on the near path: X's
// two child boxes (prune, near-first order), and if the near child N is
// interior, N's two child boxes as KIRK would test them on entering N (same
// h.t: nothing between those tests can change it).  The far child is pushed
// below N's far child, so the pops come in KIRK's order; every entry is still
// prune-tested when KIRK would pop it, and KIRK's visit counts are kept (N
// counts as a visit in the iteration that expands it).
struct WBox {
    float e0, e1, e2, x0, x1, x2;  // per-axis entry / exit (fast slab form)
};
__device__ __forceinline__ WBox wbox_fast(float mnx, float mny, float mnz, float mxx, float mxy, float mxz,
                                          const TravRay& tr) {
    const float ax = (mnx - tr.r.o.x) * tr.inv.x, bx = (mxx - tr.r.o.x) * tr.inv.x;
    const float ay = (mny - tr.r.o.y) * tr.inv.y, by = (mxy - tr.r.o.y) * tr.inv.y;
    const float az = (mnz - tr.r.o.z) * tr.inv.z, bz = (mxz - tr.r.o.z) * tr.inv.z;
    return WBox{fminf(ax, bx), fminf(ay, by), fminf(az, bz), fmaxf(ax, bx), fmaxf(ay, by), fmaxf(az, bz)};
}
__device__ __forceinline__ WBox wbox_union(const WBox& a, const WBox& b) {
    return WBox{fminf(a.e0, b.e0), fminf(a.e1, b.e1), fminf(a.e2, b.e2),
                fmaxf(a.x0, b.x0), fmaxf(a.x1, b.x1), fmaxf(a.x2, b.x2)};
}
__device__ __forceinline__ bool wbox_t(const WBox& w, float& t0, float& t1) {
    t0 = fmaxf(fmaxf(w.e0, w.e1), w.e2);
    t1 = fminf(fminf(w.x0, w.x1), w.x2);
    return t0 <= t1;
}
__device__ __forceinline__ float wmin(float a, float b) { return (b < a) ? b : a; }  // std::min, as the build
__device__ __forceinline__ float wmax(float a, float b) { return (a < b) ? b : a; }  // std::max

// One wave iteration of one lane over wide records; the leaf branch is
// iter2's.  ANY: any hit with the fixed limit tmax_any (the ray's tMax; KIRK's
// any-hit walk has the same near-first order and prune test,
// CPU_BVH.cpp:211-265), else closest hit with tlimit = h.t.  Returns true when
// the ray is finished; for ANY, `occluded` tells the result.  KIND as iter2k.
template <int KIND, bool STATS, class Stack>
__device__ __forceinline__ bool iterwk(const DevScene& S, const TravRay& tr, Hit& h, float tmax_any, Stack& stk,
                                       uint32_t& mode, Cur& c, LeafCur& lf, TravStats& st, bool& occluded,
                                       bool any_rt) {
    const bool ANY = KIND == 2 ? any_rt : KIND == 1;
    // A wave with a ray whose origin or inverse direction is not finite on
    // every axis (an exactly axis-parallel direction) runs this iteration as
    // the one-level step on the 64-B records (same entries, same stack): the
    // composed slab needs the fast form's monotone plane distances.
    if (__ballot(!tr.fin) != 0ull)
        return iter2k<KIND, STATS>(S, tr, h, tmax_any, stk, mode, c, lf, st, occluded, any_rt);
    const bool in_leaf = mode == M_LEAF;
    const bool node = mode == M_NODE;
    const bool fetch = in_leaf || node;
    const float4* p = in_leaf ? S.prims + 4 * (size_t)lf.slot : S.wide + 8 * (size_t)c.ref;
#ifdef KHP_LEAF_REUSE
    if (STATS && KIND == 0) leaf_reuse(in_leaf, lf.slot);
#endif
    float4 q0, q1, q2, q3, q4, q5, q6, q7;
    if (fetch) {
        q0 = p[0];
        q1 = p[1];
        q2 = p[2];
        q3 = p[3];
    }
    if (node) {
        q4 = p[4];
        q5 = p[5];
        q6 = p[6];
        q7 = p[7];
    }
    if (fetch) {
        pin(q0); pin(q1); pin(q2); pin(q3);
    }
    if (node) {
        pin(q4); pin(q5); pin(q6); pin(q7);
    }
    bool need_pop = mode == M_POP;
    bool have = false;
    uint32_t eref = 0u;
    float et0 = 0.0f, et1 = 0.0f;
    bool push1 = false, push2 = false;
    uint32_t p1ref = 0u, p2ref = 0u;
    float p1t0 = 0.0f, p1t1 = 0.0f, p2t0 = 0.0f, p2t1 = 0.0f;
    if (in_leaf) {
        if (STATS) st.prims++;
        if (KIND == 2) {
            float t = 0.0f;
            const bool ok = candidate_rt(q0, q1, q2, q3, tr.r, ANY, ANY ? tmax_any : lf.tmax, t);
            if (ok && ANY) {
                occluded = true;
                return true;
            }
            if (ok) {
                lf.sl = (int32_t)lf.slot;
                lf.tmax = t;
            }
        } else if (ANY) {
            if (any_candidate(q0, q1, q2, q3, tr.r, tmax_any)) {
                occluded = true;
                return true;
            }
        } else {
            leaf_candidate_t(q0, q1, q2, q3, (int32_t)lf.slot, tr.r, lf.tmax, lf.sl);
        }
        ++lf.slot;
        --lf.left;
        if (lf.left == 0u) {
            if (!ANY && lf.sl >= 0 && lf.tmax < h.t) {
                h.t = lf.tmax;
                h.slot = lf.sl;
            }
            need_pop = true;
        }
    } else if (node) {
        if (STATS) st.nodes++;
        const float tlimit = ANY ? tmax_any : h.t;
        const uint32_t c1 = __float_as_uint(q6.x), c2 = __float_as_uint(q6.y);
        const bool i1 = !ref_leaf(c1), i2 = !ref_leaf(c2);
        float gt0[4], gt1[4], At0, At1, Bt0, Bt1;
        bool gh[4], hA, hB;
        {
            const WBox w0 = wbox_fast(q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, tr);
            const WBox w1 = wbox_fast(q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, tr);
            const WBox w2 = wbox_fast(q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, tr);
            const WBox w3 = wbox_fast(q4.z, q4.w, q5.x, q5.y, q5.z, q5.w, tr);
            gh[0] = wbox_t(w0, gt0[0], gt1[0]);
            gh[1] = wbox_t(w1, gt0[1], gt1[1]);
            gh[2] = wbox_t(w2, gt0[2], gt1[2]);
            gh[3] = wbox_t(w3, gt0[3], gt1[3]);
            const WBox wa = wbox_union(w0, w1), wb = wbox_union(w2, w3);
            float ua0, ua1, ub0, ub1;
            const bool ua = wbox_t(wa, ua0, ua1), ub = wbox_t(wb, ub0, ub1);
            hA = i1 ? ua : gh[0];
            At0 = i1 ? ua0 : gt0[0];
            At1 = i1 ? ua1 : gt1[0];
            hB = i2 ? ub : gh[2];
            Bt0 = i2 ? ub0 : gt0[2];
            Bt1 = i2 ? ub1 : gt1[2];
        }
        hA = hA && !(At1 < 0.0f || At0 > tlimit);
        hB = hB && !(Bt1 < 0.0f || Bt0 > tlimit);
        const bool nearA = hA && (!hB || At0 < Bt0);  // KIRK: left first iff l0 < r0 (ties: right)
        const bool have_near = hA || hB;
        const uint32_t nref = nearA ? c1 : c2;
        const bool nint = have_near && !ref_leaf(nref);
        const bool fhit = hA && hB;
        const uint32_t fref = nearA ? c2 : c1;
        const float f0 = nearA ? Bt0 : At0, f1 = nearA ? Bt1 : At1;
        // the near child's children (tested as KIRK enters it, with the same h.t)
        const uint32_t glref = __float_as_uint(nearA ? q6.z : q7.x), grref = __float_as_uint(nearA ? q6.w : q7.y);
        const float gl0 = nearA ? gt0[0] : gt0[2], gl1 = nearA ? gt1[0] : gt1[2];
        const float gr0 = nearA ? gt0[1] : gt0[3], gr1 = nearA ? gt1[1] : gt1[3];
        const bool hl = nint && (nearA ? gh[0] : gh[2]) && !(gl1 < 0.0f || gl0 > tlimit);
        const bool hr = nint && (nearA ? gh[1] : gh[3]) && !(gr1 < 0.0f || gr0 > tlimit);
        const bool gnl = hl && (!hr || gl0 < gr0);
        const bool have_g = hl || hr;
        if (STATS && nint) st.nodes++;  // KIRK's visit of the near child
        const uint32_t gref = gnl ? glref : grref;
        const float g0 = gnl ? gl0 : gr0, g1 = gnl ? gl1 : gr1;
        // next entry: the near child (a leaf), else its near child, else the far child
        eref = !nint ? nref : (have_g ? gref : fref);
        et0 = !nint ? (nearA ? At0 : Bt0) : (have_g ? g0 : f0);
        et1 = !nint ? (nearA ? At1 : Bt1) : (have_g ? g1 : f1);
        have = have_near && (!nint || have_g || fhit);
        need_pop = !have;
        push1 = fhit && (!nint || have_g);
        p1ref = fref;
        p1t0 = f0;
        p1t1 = f1;
        push2 = hl && hr;
        p2ref = gnl ? grref : glref;
        p2t0 = gnl ? gr0 : gl0;
        p2t1 = gnl ? gr1 : gl1;
    }
    if (push1) stk.push(p1ref, p1t0, p1t1);
    if (push2) stk.push(p2ref, p2t0, p2t1);
    if (need_pop) {
        if (stk.empty()) {
            mode = M_IDLE;
            occluded = false;
            return true;
        }
        stk.pop(eref, et0, et1);
        if (et1 < 0.0f || et0 > (ANY ? tmax_any : h.t)) {
            if (STATS) st.pruned++;
            mode = M_POP;
        } else {
            have = true;
        }
    }
    if (have) take_entry<STATS>(S, eref, et0, et1, mode, c, lf, st);
    return false;
}

template <bool ANY, bool STATS, class Stack>
__device__ __forceinline__ bool iterw(const DevScene& S, const TravRay& tr, Hit& h, float tmax_any, Stack& stk,
                                      uint32_t& mode, Cur& c, LeafCur& lf, TravStats& st, bool& occluded) {
    return iterwk<ANY ? 1 : 0, STATS>(S, tr, h, tmax_any, stk, mode, c, lf, st, occluded, ANY);
}

// Whole-ray forms (batch query kernels).
template <bool STATS, class Stack>
__device__ __forceinline__ void trace_closest(const DevScene& S, const Ray& r, Hit& h, Stack& stk, TravStats& st) {
    h.t = FLT_MAX_;
    h.slot = -1;
    h.u = h.v = 0.0f;
    TravRay tr;
    trav_setup(tr, r);
    Cur c;
    if (!trav_begin(S, tr, stk, c)) return;
    while (c.valid) {
        if (ref_leaf(c.ref)) leaf_step_closest<STATS>(S, tr, h, stk, c, st);
        else interior_step<STATS>(S, tr, h.t, stk, c, st);
    }
}

template <bool STATS, class Stack>
__device__ __forceinline__ bool trace_any(const DevScene& S, const Ray& r, float tMaxRay, Stack& stk, TravStats& st) {
    TravRay tr;
    trav_setup(tr, r);
    Cur c;
    if (!trav_begin(S, tr, stk, c)) return false;
    while (c.valid) {
        if (ref_leaf(c.ref)) {
            if (leaf_step_any<STATS>(S, tr, tMaxRay, stk, c, st)) return true;
        } else {
            interior_step<STATS>(S, tr, tMaxRay, stk, c, st);
        }
    }
    return false;
}

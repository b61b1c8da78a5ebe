// bvh_build.hip -- BVH::addBaseDataStructure (CPU_BVH.cpp:16-44, 95-138, 357-552)
// on the GPU: the same binned-SAH tree, node for node and id for id, as the
// host builder in scene.cpp.
//
// KIRK's tree is defined by a sequential recursion; three facts make it a
// parallel build without changing a single node:
//   * bins, node boxes and centroid boxes are min/max/count reductions, exact
//     in any order (up to the sign of a zero);
//   * the SAH sweep over 15 planes x 3 axes is tiny and runs once per node, in
//     the host's loop order, on one thread;
//   * the Hoare two-pointer partition (CPU_BVH.cpp:475-552) swaps the k-th
//     right-belonging element of the left region with the k-th left-belonging
//     element of the right region counted from the end.  Ranking both kinds by
//     position (prefix sums) reproduces its permutation exactly.
// Nodes with more than SMALL objects are built level by level (all nodes of a
// level in one set of launches, chunks of CH objects per block); smaller nodes
// are finished by one thread each with the literal recursion.  The DFS
// preorder index of a node has a closed form,
//     pre(node) = (#left turns from the root) + 2 * (#leaves starting before node.first),
// so nodes are written straight into preorder once the leaf starts are scanned.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <chrono>
#include <string>
#include <vector>

#include "device_build.h"
#include "scene.h"

namespace khp {
namespace gb {

constexpr int NB = 16, NP = 15;
constexpr uint32_t CH = 2048;          // objects per chunk (one 256-thread block)
constexpr uint32_t SMALL = 256;        // nodes up to this many objects: one thread builds the subtree
constexpr int BW = 3 * NB * 7;         // bin words per chunk: 3 axes x 16 bins x (count, min.xyz, max.xyz)
constexpr int SUB_STACK = SMALL + 4;

struct GNode {  // interior node of the level phase
    float cb[6];
    uint32_t first, count, lturns, depth;
    int32_t axis, plane;
    float k, cbmin;
    uint32_t L, chunk0, nchunk, bad;
};
struct SRoot {  // root of a subtree finished by one thread
    float cb[6];
    uint32_t first, count, lturns, depth, n_local, pad;
};
struct LLeaf {  // leaf made by the level phase
    uint32_t first, count, lturns, depth;
};
struct Ctr {
    uint32_t n_gnode, n_sroot, n_lleaf, max_depth, max_leaf, error, pad[2];
};

// ---- box arithmetic, operand order of scene.cpp / BoundingBox.cpp ----------
struct GBox {
    float mn[3], mx[3];
};
KHD float smin(float a, float b) { return (b < a) ? b : a; }  // std::min
KHD float smax(float a, float b) { return (a < b) ? b : a; }  // std::max
KHD GBox box_empty() { return GBox{{FLT_MAX, FLT_MAX, FLT_MAX}, {-FLT_MAX, -FLT_MAX, -FLT_MAX}}; }
KHD void grow(GBox& b, const GBox& o) {
    for (int a = 0; a < 3; ++a) {
        b.mn[a] = smin(b.mn[a], o.mn[a]);
        b.mx[a] = smax(b.mx[a], o.mx[a]);
    }
}
KHD void grow_pt(GBox& b, float x, float y, float z) {
    b.mn[0] = smin(b.mn[0], x); b.mn[1] = smin(b.mn[1], y); b.mn[2] = smin(b.mn[2], z);
    b.mx[0] = smax(b.mx[0], x); b.mx[1] = smax(b.mx[1], y); b.mx[2] = smax(b.mx[2], z);
}
KHD float area(const GBox& b) {
    float sx = b.mx[0] - b.mn[0], sy = b.mx[1] - b.mn[1], sz = b.mx[2] - b.mn[2];
    return 2.0f * (sx * sy + sx * sz + sy * sz);
}
KHD bool worth(const GBox& b) {
    return b.mx[0] - b.mn[0] > 0.0f && b.mx[1] - b.mn[1] > 0.0f && b.mx[2] - b.mn[2] > 0.0f;
}
KHD float split_k(float cbmin, float cbmax) {
    const float cbdiff = cbmax - cbmin;
    const float epsilon = 0.1f;
    return ((float)NB * (1.0f - epsilon)) / cbdiff;
}
KHD GBox cb_of(const float* c) { return GBox{{c[0], c[1], c[2]}, {c[3], c[4], c[5]}}; }
KHD void cb_put(float* c, const GBox& b) {
    for (int a = 0; a < 3; ++a) {
        c[a] = b.mn[a];
        c[3 + a] = b.mx[a];
    }
}

// order-preserving float <-> uint (for min/max atomics on LDS words)
__device__ __forceinline__ uint32_t fenc(float f) {
    uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fdec(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }
__device__ __forceinline__ uint32_t bin_init(int w) {
    const int f = w % 7;
    return f == 0 ? 0u : (f <= 3 ? fenc(FLT_MAX) : fenc(-FLT_MAX));
}
__device__ __forceinline__ uint32_t bin_comb(int w, uint32_t a, uint32_t b) {
    const int f = w % 7;
    return f == 0 ? a + b : (f <= 3 ? min(a, b) : max(a, b));
}
__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// ---- setup ------------------------------------------------------------------
__global__ void k_init(const float* cen, uint32_t n, float4* rec, uint32_t* leafstart, uint32_t* part) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    __shared__ uint32_t red[6][256];
    uint32_t v[6] = {fenc(FLT_MAX), fenc(FLT_MAX), fenc(FLT_MAX), fenc(-FLT_MAX), fenc(-FLT_MAX), fenc(-FLT_MAX)};
    if (i < n) {
        const float x = cen[3 * (size_t)i], y = cen[3 * (size_t)i + 1], z = cen[3 * (size_t)i + 2];
        rec[i] = make_float4(x, y, z, __uint_as_float(i));
        v[0] = fenc(x); v[1] = fenc(y); v[2] = fenc(z);
        v[3] = v[0]; v[4] = v[1]; v[5] = v[2];
    }
    if (i <= n) leafstart[i] = 0u;
    for (int a = 0; a < 6; ++a) red[a][threadIdx.x] = v[a];
    __syncthreads();
    for (uint32_t w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int a = 0; a < 6; ++a) {
                uint32_t o = red[a][threadIdx.x + w];
                red[a][threadIdx.x] = a < 3 ? min(red[a][threadIdx.x], o) : max(red[a][threadIdx.x], o);
            }
        __syncthreads();
    }
    if (threadIdx.x < 6) part[6 * blockIdx.x + threadIdx.x] = red[threadIdx.x][0];
}

// ---- level phase ------------------------------------------------------------
__global__ void k_nchunks(const GNode* g, uint32_t b, uint32_t n, uint32_t* nc) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) nc[i] = (g[b + i].count + CH - 1) / CH;
    if (i == n) nc[i] = 0;
}

__global__ void k_chunk_list(GNode* g, uint32_t b, const uint32_t* c0, uint32_t* chunk_node) {
    const uint32_t i = blockIdx.x;
    const uint32_t base = c0[i], nc = c0[i + 1] - base;
    if (threadIdx.x == 0) {
        g[b + i].chunk0 = base;
        g[b + i].nchunk = nc;
    }
    for (uint32_t j = threadIdx.x; j < nc; j += blockDim.x) chunk_node[base + j] = b + i;
}

// Per chunk: the 3 x 16 bins of BVHNode::partition's first loop (CPU_BVH.cpp:369-399).
__global__ __launch_bounds__(256) void k_bin(const float4* __restrict__ rec, const GNode* __restrict__ g,
                                             const uint32_t* __restrict__ chunk_node, uint32_t* __restrict__ part) {
    __shared__ uint32_t tab[4][BW];
    const uint32_t c = blockIdx.x, wave = threadIdx.x >> 6;
    for (int w = threadIdx.x; w < 4 * BW; w += 256) tab[w / BW][w % BW] = bin_init(w % BW);
    const GNode nd = g[chunk_node[c]];
    const uint32_t start = nd.first + (c - nd.chunk0) * CH;
    const uint32_t end = min(nd.first + nd.count, start + CH);
    float k[3], cbmin[3];
    for (int a = 0; a < 3; ++a) {
        cbmin[a] = nd.cb[a];
        k[a] = split_k(nd.cb[a], nd.cb[3 + a]);
    }
    __syncthreads();
    for (uint32_t p = start + threadIdx.x; p < end; p += 256) {
        const float4 e = rec[p];
        const float cc[3] = {e.x, e.y, e.z};
        const uint32_t ex = fenc(e.x), ey = fenc(e.y), ez = fenc(e.z);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const int bin = min(max((int)(k[a] * (cc[a] - cbmin[a])), 0), NB - 1);  // in range for valid input
            uint32_t* t = &tab[wave][(a * NB + bin) * 7];
            atomicAdd(&t[0], 1u);
            atomicMin(&t[1], ex);
            atomicMin(&t[2], ey);
            atomicMin(&t[3], ez);
            atomicMax(&t[4], ex);
            atomicMax(&t[5], ey);
            atomicMax(&t[6], ez);
        }
    }
    __syncthreads();
    for (int w = threadIdx.x; w < BW; w += 256) {
        uint32_t v = tab[0][w];
        for (int q = 1; q < 4; ++q) v = bin_comb(w, v, tab[q][w]);
        part[(size_t)c * BW + w] = v;
    }
}

__device__ void spawn(uint32_t first, uint32_t count, const GBox& cb, uint32_t lturns, uint32_t depth, GNode* g,
                      uint32_t gcap, SRoot* sr, uint32_t scap, LLeaf* ll, uint32_t lcap, uint32_t* leafstart, Ctr* ct) {
    atomicMax(&ct->max_depth, depth);
    if (count - 1u > 1u && worth(cb)) {
        if (count <= SMALL) {
            const uint32_t s = atomicAdd(&ct->n_sroot, 1u);
            if (s >= scap) { atomicOr(&ct->error, 1u); return; }
            SRoot r{};
            cb_put(r.cb, cb);
            r.first = first; r.count = count; r.lturns = lturns; r.depth = depth;
            sr[s] = r;
        } else {
            const uint32_t s = atomicAdd(&ct->n_gnode, 1u);
            if (s >= gcap) { atomicOr(&ct->error, 2u); return; }
            GNode q{};
            cb_put(q.cb, cb);
            q.first = first; q.count = count; q.lturns = lturns; q.depth = depth;
            q.plane = -1;
            g[s] = q;
        }
    } else {
        const uint32_t s = atomicAdd(&ct->n_lleaf, 1u);
        if (s >= lcap) { atomicOr(&ct->error, 4u); return; }
        ll[s] = LLeaf{first, count, lturns, depth};
        leafstart[first] = 1u;
        atomicMax(&ct->max_leaf, count);
    }
}

// Per node: reduce the chunk bins, run the SAH sweep exactly as the host loop
// (CPU_BVH.cpp:400-470), spawn the two children.
// The SAH sweep of one axis over its 16 encoded bins (t: 16 x 7 words), in
// the host loop's order and arithmetic (CPU_BVH.cpp:400-470, scene.cpp
// Builder::partition): left prefix boxes, then planes 14 .. 0 with the right
// suffix, strict <.  lbw: 15 x 7 words of scratch (LDS).
struct AxisBest {
    float best;
    int plane;
    uint32_t L;
    GBox lcb, rcb;
};
__device__ __forceinline__ GBox bin_box(const uint32_t* t) {
    return GBox{{fdec(t[1]), fdec(t[2]), fdec(t[3])}, {fdec(t[4]), fdec(t[5]), fdec(t[6])}};
}
__device__ AxisBest sweep_axis(const uint32_t* t, float* lbw) {
    GBox acc = box_empty();
    uint32_t cnt = 0;
#pragma unroll 1
    for (int p = 0; p < NP; ++p) {
        GBox l = box_empty();
        if (p > 0) grow(l, acc);
        grow(l, bin_box(t + 7 * p));
        acc = l;
        cnt += t[7 * p];
        float* o = lbw + 7 * p;
        o[0] = __uint_as_float(cnt);
        for (int a = 0; a < 3; ++a) {
            o[1 + a] = acc.mn[a];
            o[4 + a] = acc.mx[a];
        }
    }
    AxisBest r{FLT_MAX, 0, 0u, box_empty(), box_empty()};
    GBox rb_next = box_empty();
    uint32_t rn_next = 0;
#pragma unroll 1
    for (int p = NP - 1; p >= 0; --p) {
        GBox rb = box_empty();
        grow(rb, bin_box(t + 7 * (p + 1)));
        uint32_t rn = t[7 * (p + 1)];
        if (p != NP - 1) {
            grow(rb, rb_next);
            rn += rn_next;
        }
        const float* o = lbw + 7 * p;
        const GBox lb{{o[1], o[2], o[3]}, {o[4], o[5], o[6]}};
        const uint32_t ln = __float_as_uint(o[0]);
        const float cost = area(lb) * (float)ln + area(rb) * (float)rn;
        if (cost < r.best) {
            r.best = cost;
            r.plane = p;
            r.L = ln;
            r.lcb = lb;
            r.rcb = rb;
        }
        rb_next = rb;
        rn_next = rn;
    }
    return r;
}

constexpr int PICK_GROUPS = 3;  // 3 x 336 threads reduce every 3rd chunk each

__global__ __launch_bounds__(PICK_GROUPS * BW) void k_pick(GNode* g, uint32_t b, const uint32_t* __restrict__ part,
                                                           uint32_t gcap, SRoot* sr, uint32_t scap, LLeaf* ll,
                                                           uint32_t lcap, uint32_t* leafstart, Ctr* ct) {
    __shared__ uint32_t red[PICK_GROUPS][BW];
    const uint32_t i = b + blockIdx.x;
    const uint32_t c0 = g[i].chunk0, nc = g[i].nchunk;
    {
        const int w = (int)(threadIdx.x % BW), grp = (int)(threadIdx.x / BW);
        uint32_t v = bin_init(w);
        uint32_t c = c0 + grp;
        for (; c + 3 * PICK_GROUPS < c0 + nc; c += 4 * PICK_GROUPS) {  // 4 independent loads in flight
            const uint32_t a0 = part[(size_t)c * BW + w];
            const uint32_t a1 = part[(size_t)(c + PICK_GROUPS) * BW + w];
            const uint32_t a2 = part[(size_t)(c + 2 * PICK_GROUPS) * BW + w];
            const uint32_t a3 = part[(size_t)(c + 3 * PICK_GROUPS) * BW + w];
            v = bin_comb(w, bin_comb(w, v, a0), bin_comb(w, bin_comb(w, a1, a2), a3));
        }
        for (; c < c0 + nc; c += PICK_GROUPS) v = bin_comb(w, v, part[(size_t)c * BW + w]);
        red[grp][w] = v;
    }
    __syncthreads();
    for (int w = threadIdx.x; w < BW; w += blockDim.x)
        for (int q = 1; q < PICK_GROUPS; ++q) red[0][w] = bin_comb(w, red[0][w], red[q][w]);
    __syncthreads();
    if (threadIdx.x != 0) return;
    GNode nd = g[i];
    __shared__ float lbw[NP * 7];
    float best = FLT_MAX;
    int best_axis = 0, best_plane = 0;
    uint32_t bestL = 0;
    GBox lcb = box_empty(), rcb = box_empty();
    for (int axis = 0; axis < 3; ++axis) {
        const AxisBest r = sweep_axis(&red[0][axis * NB * 7], lbw);
        if (r.best < best) {
            best = r.best;
            best_axis = axis;
            best_plane = r.plane;
            bestL = r.L;
            lcb = r.lcb;
            rcb = r.rcb;
        }
    }
    nd.axis = best_axis;
    nd.plane = best_plane;
    nd.cbmin = nd.cb[best_axis];
    nd.k = split_k(nd.cb[best_axis], nd.cb[3 + best_axis]);
    nd.L = bestL;
    if (bestL == 0 || bestL >= nd.count) {  // cannot happen for worth(cb) boxes; refuse rather than loop
        nd.bad = 1;
        atomicOr(&ct->error, 8u);
    }
    g[i] = nd;
    if (nd.bad) return;
    spawn(nd.first, bestL, lcb, nd.lturns + 1, nd.depth + 1, g, gcap, sr, scap, ll, lcap, leafstart, ct);
    spawn(nd.first + bestL, nd.count - bestL, rcb, nd.lturns, nd.depth + 1, g, gcap, sr, scap, ll, lcap, leafstart, ct);
}

__device__ __forceinline__ bool right_side(const GNode& nd, float4 e) {
    const float c = nd.axis == 0 ? e.x : (nd.axis == 1 ? e.y : e.z);
    return (int)(nd.k * (c - nd.cbmin)) > nd.plane;
}

// Per chunk: count right-belonging objects in the left region and left-belonging
// objects in the right region.  (hi 32 bits, lo 32 bits)
__global__ __launch_bounds__(256) void k_classify(const float4* __restrict__ rec, const GNode* __restrict__ g,
                                                  const uint32_t* __restrict__ chunk_node, uint64_t* cnt) {
    __shared__ uint32_t sL, sR;
    if (threadIdx.x == 0) sL = sR = 0;
    __syncthreads();
    const uint32_t c = blockIdx.x;
    const GNode nd = g[chunk_node[c]];
    const uint32_t start = nd.first + (c - nd.chunk0) * CH;
    const uint32_t end = min(nd.first + nd.count, start + CH);
    const uint32_t mid = nd.first + nd.L;
    uint32_t l = 0, r = 0;
    if (!nd.bad)
        for (uint32_t p = start + threadIdx.x; p < end; p += 256) {
            const bool rs = right_side(nd, rec[p]);
            l += (p < mid && rs);
            r += (p >= mid && !rs);
        }
    if (l) atomicAdd(&sL, l);
    if (r) atomicAdd(&sR, r);
    __syncthreads();
    if (threadIdx.x == 0) cnt[c] = ((uint64_t)sL << 32) | sR;
    if (threadIdx.x == 0 && c == gridDim.x - 1) cnt[c + 1] = 0;
}

// Per chunk: rank the misplaced objects by position and stage the swap pairs.
__global__ __launch_bounds__(256) void k_swap_write(const float4* __restrict__ rec, const GNode* __restrict__ g,
                                                    const uint32_t* __restrict__ chunk_node, const uint64_t* off,
                                                    float4* SL, float4* SR, uint32_t* PL, uint32_t* PR) {
    __shared__ uint32_t wl[4], wr[4];
    const uint32_t c = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const GNode nd = g[chunk_node[c]];
    if (nd.bad) return;
    const uint32_t start = nd.first + (c - nd.chunk0) * CH;
    const uint32_t end = min(nd.first + nd.count, start + CH);
    const uint32_t mid = nd.first + nd.L;
    const uint64_t o0 = off[nd.chunk0], oc = off[c], oe = off[nd.chunk0 + nd.nchunk];
    uint32_t baseL = (uint32_t)(oc >> 32) - (uint32_t)(o0 >> 32);
    uint32_t baseR = (uint32_t)oc - (uint32_t)o0;
    const uint32_t mR = (uint32_t)oe - (uint32_t)o0;
    (void)lane;
    for (uint32_t r0 = start; r0 < end; r0 += 256) {
        const uint32_t p = r0 + threadIdx.x;
        float4 e = make_float4(0, 0, 0, 0);
        bool fl = false, fr = false;
        if (p < end) {
            e = rec[p];
            const bool rs = right_side(nd, e);
            fl = p < mid && rs;
            fr = p >= mid && !rs;
        }
        const uint64_t bl = __ballot(fl), br = __ballot(fr);
        if ((threadIdx.x & 63) == 0) {
            wl[wave] = (uint32_t)__popcll(bl);
            wr[wave] = (uint32_t)__popcll(br);
        }
        __syncthreads();
        uint32_t pl = baseL, pr = baseR, tl = 0, tr = 0;
        for (uint32_t q = 0; q < 4; ++q) {
            if (q < wave) { pl += wl[q]; pr += wr[q]; }
            tl += wl[q];
            tr += wr[q];
        }
        if (fl) {
            const uint32_t kk = pl + lane_rank(bl);
            SL[nd.first + kk] = e;
            PL[nd.first + kk] = p;
        }
        if (fr) {
            const uint32_t kk = mR - 1u - (pr + lane_rank(br));
            SR[nd.first + kk] = e;
            PR[nd.first + kk] = p;
        }
        baseL += tl;
        baseR += tr;
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_swap_apply(float4* rec, const GNode* __restrict__ g,
                                                    const uint32_t* __restrict__ chunk_node, const uint64_t* off,
                                                    const float4* SL, const float4* SR, const uint32_t* PL,
                                                    const uint32_t* PR) {
    const uint32_t c = blockIdx.x;
    const GNode nd = g[chunk_node[c]];
    if (nd.bad) return;
    const uint32_t m = (uint32_t)(off[nd.chunk0 + nd.nchunk] >> 32) - (uint32_t)(off[nd.chunk0] >> 32);
    const uint32_t start = (c - nd.chunk0) * CH;
    const uint32_t end = min(m, start + CH);
    for (uint32_t kk = start + threadIdx.x; kk < end; kk += 256) {
        const uint32_t s = nd.first + kk;
        rec[PL[s]] = SR[s];
        rec[PR[s]] = SL[s];
    }
}

// ---- small subtrees: the literal recursion of BVHNode::split, one thread each ----
struct Frame {
    float cb[6];
    uint32_t first, second, depth;
    int32_t parent;  // local index of the parent, -1 for the subtree root
    int32_t side;
};

// Values every lane of the wave holds identically, made scalar for the compiler
// so that the loops and branches on them stay wave-uniform (the subtree kernel
// relies on the wave moving through its steps together).
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int32_t uni(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float uni(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

__device__ __forceinline__ float wave_min(float v) {
    for (int o = 32; o > 0; o >>= 1) v = smin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
    for (int o = 32; o > 0; o >>= 1) v = smax(v, __shfl_xor(v, o));
    return v;
}

// One wave per subtree (persistent blocks pull subtrees from a counter): the
// node range lives in LDS; per node the lanes reduce the box, fill the 3 x 16
// bins with LDS atomics, three lanes sweep one axis each, and the Hoare pairs
// of the partition are ranked with ballots and swapped in LDS.  The nodes come
// out in the recursion's preorder (explicit stack, left child popped first).
__global__ __launch_bounds__(64) void k_subtree(float4* rec, const float* __restrict__ bounds, SRoot* sr, uint32_t n,
                                                uint32_t* next, BuildNode* T, uint32_t* leafstart, Ctr* ct,
                                                Frame* fstack) {
    __shared__ float4 srec[SMALL];
    __shared__ float sb[6][SMALL];
    __shared__ uint32_t bins[BW];
    __shared__ uint32_t PL[SMALL / 2 + 1], PR[SMALL / 2 + 1];
    __shared__ float s_lcb[1][6], s_rcb[1][6];
    const uint32_t lane = threadIdx.x;
    Frame* stk = fstack + (size_t)blockIdx.x * SUB_STACK;
    // every lane runs the atomic (no branch), lane 0 adds the 1: its old value is
    // the wave's ticket, made scalar so the loop below is wave-uniform
    uint32_t si = uni(atomicAdd(next, lane == 0 ? 1u : 0u));
    while (si < n) {
        const SRoot root = sr[si];
        const uint32_t base = uni(root.first), cnt = uni(root.count);
        for (uint32_t i = lane; i < cnt; i += 64) {
            const float4 e = rec[base + i];
            srec[i] = e;
            const float* bb = bounds + 6 * (size_t)__float_as_uint(e.w);
            for (int q = 0; q < 6; ++q) sb[q][i] = bb[q];
        }
        BuildNode* out = T + 2 * (size_t)base;
        if (lane == 0) {
            Frame f{};
            for (int q = 0; q < 6; ++q) f.cb[q] = root.cb[q];
            f.first = 0;
            f.second = cnt - 1;
            f.depth = root.depth;
            f.parent = -1;
            f.side = 0;
            stk[0] = f;
        }
        int sp = 1;
        int32_t local = 0;
        uint32_t maxd = 0, maxl = 0;
        bool failed = false;
        while (sp > 0 && !failed) {
            __syncthreads();
            Frame f = stk[--sp];
            for (int q = 0; q < 6; ++q) f.cb[q] = uni(f.cb[q]);
            f.first = uni(f.first);
            f.second = uni(f.second);
            f.depth = uni(f.depth);
            f.parent = uni(f.parent);
            f.side = uni(f.side);
            const int32_t ni = local++;
            if (ni >= 2 * (int32_t)cnt) {  // a subtree of cnt objects has < 2 cnt nodes: never spin
                if (lane == 0) atomicOr(&ct->error, 64u);
                failed = true;
                break;
            }
#ifdef KHP_BUILD_DEBUG
            if (lane == 0)
                printf("sub %u sp %d ni %d first %u second %u depth %u parent %d side %d cb %g %g %g %g %g %g\n", si, sp,
                       ni, f.first, f.second, f.depth, f.parent, f.side, f.cb[0], f.cb[1], f.cb[2], f.cb[3], f.cb[4],
                       f.cb[5]);
#endif
            if (lane == 0 && f.parent >= 0) {
                if (f.side == 0) out[f.parent].left = ni;
                else out[f.parent].right = ni;
            }
            float bmn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, bmx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
            for (uint32_t i = f.first + lane; i <= f.second; i += 64)
                for (int a = 0; a < 3; ++a) {
                    bmn[a] = smin(bmn[a], sb[a][i]);
                    bmx[a] = smax(bmx[a], sb[3 + a][i]);
                }
            BuildNode node{};
            node.mn = mk(wave_min(bmn[0]), wave_min(bmn[1]), wave_min(bmn[2]));
            node.mx = mk(wave_max(bmx[0]), wave_max(bmx[1]), wave_max(bmx[2]));
            maxd = max(maxd, f.depth);
            const GBox cb = cb_of(f.cb);
            const uint32_t c = f.second - f.first + 1;
            if (c - 1u > 1u && worth(cb)) {
                float k[3], cbmin[3];
                for (int a = 0; a < 3; ++a) {
                    cbmin[a] = cb.mn[a];
                    k[a] = split_k(cb.mn[a], cb.mx[a]);
                }
                for (int w = lane; w < BW; w += 64) bins[w] = bin_init(w);
                __syncthreads();
                for (uint32_t i = f.first + lane; i <= f.second; i += 64) {
                    const float4 e = srec[i];
                    const float cc[3] = {e.x, e.y, e.z};
                    const uint32_t ex = fenc(e.x), ey = fenc(e.y), ez = fenc(e.z);
                    for (int a = 0; a < 3; ++a) {
                        const int bin = min(max((int)(k[a] * (cc[a] - cbmin[a])), 0), NB - 1);
                        uint32_t* t = &bins[(a * NB + bin) * 7];
                        atomicAdd(&t[0], 1u);
                        atomicMin(&t[1], ex);
                        atomicMin(&t[2], ey);
                        atomicMin(&t[3], ez);
                        atomicMax(&t[4], ex);
                        atomicMax(&t[5], ey);
                        atomicMax(&t[6], ez);
                    }
                }
                __syncthreads();
                // SAH sweep on 48 lanes: lane = axis * 16 + bin.  Prefix (left) and
                // suffix (right) unions by segmented shuffles, one (axis, plane)
                // cost per lane, then the host loop's choice: the first strict
                // minimum in the order axis 0..2, plane 14..0, below FLT_MAX.
                const int sax = (int)(lane >> 4), sb16 = (int)(lane & 15);
                GBox lb = box_empty(), rb = box_empty();
                uint32_t ln = 0, rn = 0;
                if (sax < 3) {
                    const uint32_t* t = &bins[(sax * NB + sb16) * 7];
                    lb = bin_box(t);
                    rb = lb;
                    ln = rn = t[0];
                }
                for (int d = 1; d < 16; d <<= 1) {
                    GBox ol, orr;
                    for (int q = 0; q < 3; ++q) {
                        ol.mn[q] = __shfl_up(lb.mn[q], d, 16);
                        ol.mx[q] = __shfl_up(lb.mx[q], d, 16);
                        orr.mn[q] = __shfl_down(rb.mn[q], d, 16);
                        orr.mx[q] = __shfl_down(rb.mx[q], d, 16);
                    }
                    const uint32_t oln = __shfl_up(ln, d, 16), orn = __shfl_down(rn, d, 16);
                    if (sb16 >= d) {  // left prefix: bins 0..b (earlier bins first, as the host's grow chain)
                        GBox m = box_empty();
                        grow(m, ol);
                        grow(m, lb);
                        lb = m;
                        ln += oln;
                    }
                    if (sb16 + d < 16) {  // right suffix: bins b..15
                        GBox m = box_empty();
                        grow(m, rb);
                        grow(m, orr);
                        rb = m;
                        rn += orn;
                    }
                }
                // plane p = b: left = bins 0..p, right = bins p+1..15
                GBox rb1;
                for (int q = 0; q < 3; ++q) {
                    rb1.mn[q] = __shfl_down(rb.mn[q], 1, 16);
                    rb1.mx[q] = __shfl_down(rb.mx[q], 1, 16);
                }
                const uint32_t rn1 = __shfl_down(rn, 1, 16);
                float cost = area(lb) * (float)ln + area(rb1) * (float)rn1;
                const bool valid = sax < 3 && sb16 < NP && cost < FLT_MAX;
                uint32_t order = valid ? (uint32_t)(sax * NP + (NP - 1 - sb16)) : 0xffffffffu;
                if (!valid) cost = FLT_MAX;
                float bc = cost;
                uint32_t bo = order;
                for (int o = 32; o > 0; o >>= 1) {
                    const float oc = __shfl_xor(bc, o);
                    const uint32_t oo = __shfl_xor(bo, o);
                    if (oc < bc || (oc == bc && oo < bo)) {
                        bc = oc;
                        bo = oo;
                    }
                }
                bo = uni(bo);
                const bool found = bo != 0xffffffffu;
                const int ax = found ? (int)(bo / NP) : 0;
                const int plane = found ? (NP - 1) - (int)(bo % NP) : 0;
                const int win = ax * 16 + plane;
                const uint32_t L = found ? uni((uint32_t)__shfl(ln, win)) : 0u;
                if (lane == (uint32_t)win && found) {
                    cb_put(s_lcb[0], lb);
                    cb_put(s_rcb[0], rb1);
                }
                __syncthreads();
                if (L == 0 || L >= c) {  // cannot happen for worth(cb) boxes; refuse rather than loop
                    if (lane == 0) atomicOr(&ct->error, 32u);
                    failed = true;
                    break;
                }
                const uint32_t mid = f.first + L;
#ifdef KHP_BUILD_DEBUG
                if (lane == 0) printf("  split ax %d plane %d L %u cost %g\n", ax, plane, L, bc);
#endif
                uint32_t mL = 0, mR = 0;
                for (uint32_t r0 = f.first; r0 <= f.second; r0 += 64) {
                    const uint32_t i = r0 + lane;
                    bool fl = false, fr = false;
                    if (i <= f.second) {
                        const float4 e = srec[i];
                        const float cc = ax == 0 ? e.x : (ax == 1 ? e.y : e.z);
                        const bool rs = (int)(k[ax] * (cc - cbmin[ax])) > plane;
                        fl = i < mid && rs;
                        fr = i >= mid && !rs;
                    }
                    const uint64_t bl = __ballot(fl), br = __ballot(fr);
                    if (fl) PL[mL + lane_rank(bl)] = i;
                    if (fr) PR[mR + lane_rank(br)] = i;
                    mL += (uint32_t)__popcll(bl);
                    mR += (uint32_t)__popcll(br);
                }
                __syncthreads();
                // k-th misplaced of the left region <-> k-th misplaced of the right region from its end
                for (uint32_t q = lane; q < mL; q += 64) {
                    const uint32_t pa = PL[q], pb = PR[mR - 1u - q];
                    const float4 ta = srec[pa];
                    srec[pa] = srec[pb];
                    srec[pb] = ta;
                    for (int z = 0; z < 6; ++z) {
                        const float tz = sb[z][pa];
                        sb[z][pa] = sb[z][pb];
                        sb[z][pb] = tz;
                    }
                }
                if (lane == 0) {
                    node.count = 0;
                    out[ni] = node;
                }
                if (sp + 2 > SUB_STACK) {
                    if (lane == 0) atomicOr(&ct->error, 16u);
                    failed = true;
                    break;
                }
                GBox lcb = box_empty(), rcb = box_empty();
                if (found) {
                    lcb = cb_of(s_lcb[0]);
                    rcb = cb_of(s_rcb[0]);
                }
                if (lane == 0) {
                    Frame r{};
                    cb_put(r.cb, rcb);
                    r.first = mid; r.second = f.second; r.depth = f.depth + 1; r.parent = ni; r.side = 1;
                    stk[sp] = r;
                    Frame l{};
                    cb_put(l.cb, lcb);
                    l.first = f.first; l.second = mid - 1; l.depth = f.depth + 1; l.parent = ni; l.side = 0;
                    stk[sp + 1] = l;
                }
                sp += 2;
            } else {
                node.first = (int32_t)(base + f.first);
                node.count = (int32_t)c;
                node.left = node.right = -1;
                if (lane == 0) {
                    out[ni] = node;
                    leafstart[base + f.first] = 1u;
                }
                maxl = max(maxl, c);
            }
        }
        __syncthreads();
        for (uint32_t i = lane; i < cnt; i += 64) rec[base + i] = srec[i];
        if (lane == 0) {
            sr[si].n_local = (uint32_t)local;
            atomicMax(&ct->max_depth, maxd);
            atomicMax(&ct->max_leaf, maxl);
        }
        si = uni(atomicAdd(next, lane == 0 ? 1u : 0u));
    }
}

// ---- assembly into DFS preorder ---------------------------------------------
__global__ void k_copy_subtrees(const SRoot* sr, uint32_t n, const BuildNode* T, const uint32_t* P, BuildNode* fin) {
    const uint32_t si = blockIdx.x * blockDim.x + threadIdx.x;
    if (si >= n) return;
    const SRoot r = sr[si];
    const int32_t pre = (int32_t)(r.lturns + 2u * P[r.first]);
    const BuildNode* src = T + 2 * (size_t)r.first;
    for (uint32_t j = 0; j < r.n_local; ++j) {
        BuildNode nd = src[j];
        if (nd.count == 0) {
            nd.left += pre;
            nd.right += pre;
        }
        fin[pre + j] = nd;
    }
}

__global__ void k_level_leaves(const LLeaf* ll, uint32_t n, const float4* rec, const float* bounds, const uint32_t* P,
                               BuildNode* fin) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const LLeaf l = ll[i];
    GBox bv = box_empty();
    for (uint32_t id = l.first; id < l.first + l.count; ++id) {
        const float* bb = &bounds[6 * (size_t)__float_as_uint(rec[id].w)];
        bv.mn[0] = smin(bv.mn[0], bb[0]); bv.mn[1] = smin(bv.mn[1], bb[1]); bv.mn[2] = smin(bv.mn[2], bb[2]);
        bv.mx[0] = smax(bv.mx[0], bb[3]); bv.mx[1] = smax(bv.mx[1], bb[4]); bv.mx[2] = smax(bv.mx[2], bb[5]);
    }
    BuildNode nd{};
    nd.mn = mk(bv.mn[0], bv.mn[1], bv.mn[2]);
    nd.mx = mk(bv.mx[0], bv.mx[1], bv.mx[2]);
    nd.left = nd.right = -1;
    nd.first = (int32_t)l.first;
    nd.count = (int32_t)l.count;
    fin[l.lturns + 2u * P[l.first]] = nd;
}

__global__ void k_level_interior(const GNode* g, uint32_t b, uint32_t n, const uint32_t* P, BuildNode* fin) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const GNode nd = g[b + i];
    const int32_t pre = (int32_t)(nd.lturns + 2u * P[nd.first]);
    const int32_t l = pre + 1;
    const int32_t r = pre + 2 * (int32_t)(P[nd.first + nd.L] - P[nd.first]);
    const BuildNode L = fin[l], R = fin[r];
    GBox bv = box_empty();
    grow(bv, GBox{{L.mn.x, L.mn.y, L.mn.z}, {L.mx.x, L.mx.y, L.mx.z}});
    grow(bv, GBox{{R.mn.x, R.mn.y, R.mn.z}, {R.mx.x, R.mx.y, R.mx.z}});
    BuildNode o{};
    o.mn = mk(bv.mn[0], bv.mn[1], bv.mn[2]);
    o.mx = mk(bv.mx[0], bv.mx[1], bv.mx[2]);
    o.left = l;
    o.right = r;
    o.first = 0;
    o.count = 0;
    fin[pre] = o;
}

__global__ void k_ids(const float4* rec, uint32_t n, uint32_t* ids) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ids[i] = __float_as_uint(rec[i].w);
}

// ---- host driver --------------------------------------------------------------
struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
    ~Buf() {
        if (p) (void)hipFree(p);
    }
    hipError_t ensure(size_t n) {
        if (n <= bytes && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, n ? n : 16);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    // grow keeping the first `keep` bytes
    hipError_t grow(size_t n, size_t keep, hipStream_t s) {
        if (n <= bytes && p) return hipSuccess;
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, n);
        if (e != hipSuccess) return e;
        if (p && keep) e = hipMemcpyAsync(q, p, keep, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
        if (p) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(p);
        }
        p = q;
        bytes = n;
        return hipSuccess;
    }
    template <typename T>
    T* as() const { return (T*)p; }
};

#define GBCHK(expr)                                                                  \
    do {                                                                             \
        hipError_t e_ = (expr);                                                      \
        if (e_ != hipSuccess) return std::string(#expr) + ": " + hipGetErrorString(e_); \
    } while (0)

static uint32_t blocks(uint64_t n, uint32_t b) { return (uint32_t)((n + b - 1) / b); }

}  // namespace gb

// Builds the DFS-preorder tree of build_bvh() on the device from hs.centroid /
// hs.bounds into t; sets hs.depth, hs.max_leaf.  Returns an error string.
std::string device_build_bvh(HostScene& hs, const DeviceObjects& o, hipStream_t st, DeviceTree& t,
                             double* kernel_ms) {
    using namespace gb;
    const uint32_t N = o.n_obj;
    if (N == 0) return "no objects";
    auto t0 = std::chrono::steady_clock::now();
    Buf rec, leafstart, part0;
    const float* cen = o.centroid.as<float>();
    const float* bnd = o.bounds.as<float>();
    GBCHK(rec.ensure(16 * (size_t)N));
    GBCHK(leafstart.ensure(4 * ((size_t)N + 1)));
    const uint32_t nb0 = blocks(N + 1, 256);
    GBCHK(part0.ensure(24 * (size_t)nb0));
    hipLaunchKernelGGL(k_init, dim3(nb0), dim3(256), 0, st, cen, N, rec.as<float4>(),
                       leafstart.as<uint32_t>(), part0.as<uint32_t>());
    GBCHK(hipGetLastError());
    hipEvent_t ev0, ev1;
    GBCHK(hipEventCreate(&ev0));
    GBCHK(hipEventCreate(&ev1));
    GBCHK(hipEventRecord(ev0, st));
    std::vector<uint32_t> hp(6 * (size_t)nb0);
    GBCHK(hipMemcpyAsync(hp.data(), part0.p, hp.size() * 4, hipMemcpyDeviceToHost, st));
    GBCHK(hipStreamSynchronize(st));
    auto dec = [](uint32_t u) {
        uint32_t b = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
        float f;
        memcpy(&f, &b, 4);
        return f;
    };
    uint32_t red[6] = {hp[0], hp[1], hp[2], hp[3], hp[4], hp[5]};
    for (uint32_t b = 1; b < nb0; ++b)
        for (int a = 0; a < 6; ++a) red[a] = a < 3 ? std::min(red[a], hp[6 * b + a]) : std::max(red[a], hp[6 * b + a]);
    GBox rootcb;
    for (int a = 0; a < 3; ++a) {
        rootcb.mn[a] = dec(red[a]);
        rootcb.mx[a] = dec(red[3 + a]);
    }

    // scratch of the level phase, grown on demand
    Buf gn, srb, llb, ctr, nc, c0, chunk_node, part, cnt, off, SL, SR, PL, PR, tmp;
    size_t gcap = 1024, scap = 1024, lcap = 1024;
    GBCHK(gn.ensure(gcap * sizeof(GNode)));
    GBCHK(srb.ensure(scap * sizeof(SRoot)));
    GBCHK(llb.ensure(lcap * sizeof(LLeaf)));
    GBCHK(ctr.ensure(sizeof(Ctr)));
    Ctr hc{};
    // the root: KIRK's split() on (0, N-1) with the centroid box of everything
    const bool root_split = (N - 1u > 1u) && worth(rootcb);
    if (root_split && N > SMALL) {
        GNode r{};
        cb_put(r.cb, rootcb);
        r.first = 0; r.count = N; r.lturns = 0; r.depth = 1; r.plane = -1;
        GBCHK(hipMemcpyAsync(gn.p, &r, sizeof(r), hipMemcpyHostToDevice, st));
        hc.n_gnode = 1;
    } else if (root_split) {
        SRoot r{};
        cb_put(r.cb, rootcb);
        r.first = 0; r.count = N; r.lturns = 0; r.depth = 1;
        GBCHK(hipMemcpyAsync(srb.p, &r, sizeof(r), hipMemcpyHostToDevice, st));
        hc.n_sroot = 1;
    } else {
        LLeaf l{0, N, 0, 1};
        GBCHK(hipMemcpyAsync(llb.p, &l, sizeof(l), hipMemcpyHostToDevice, st));
        const uint32_t one = 1;
        GBCHK(hipMemcpyAsync(leafstart.p, &one, 4, hipMemcpyHostToDevice, st));
        hc.n_lleaf = 1;
        hc.max_leaf = N;
    }
    hc.max_depth = 1;
    GBCHK(hipMemcpyAsync(ctr.p, &hc, sizeof(hc), hipMemcpyHostToDevice, st));
    // hipcub scratch
    size_t tb1 = 0, tb2 = 0;
    GBCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb1, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)N + 2, st));
    GBCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb2, (uint64_t*)nullptr, (uint64_t*)nullptr, (int)N + 2, st));
    GBCHK(tmp.ensure(std::max(tb1, tb2)));
    GBCHK(SL.ensure(16 * (size_t)N));
    GBCHK(SR.ensure(16 * (size_t)N));
    GBCHK(PL.ensure(4 * (size_t)N));
    GBCHK(PR.ensure(4 * (size_t)N));
    std::vector<std::pair<uint32_t, uint32_t>> levels;  // (begin, count) in gn
    uint32_t lb = 0, le = hc.n_gnode;
    while (le > lb) {
        const uint32_t n = le - lb;
        levels.emplace_back(lb, n);
        // children of this level: at most 2 per node in each list
        if (le + 2 * (size_t)n > gcap) {
            size_t nc2 = std::max(gcap * 2, (size_t)le + 2 * n);
            GBCHK(gn.grow(nc2 * sizeof(GNode), (size_t)le * sizeof(GNode), st));
            gcap = nc2;
        }
        if (hc.n_sroot + 2 * (size_t)n > scap) {
            size_t nc2 = std::max(scap * 2, (size_t)hc.n_sroot + 2 * n);
            GBCHK(srb.grow(nc2 * sizeof(SRoot), (size_t)hc.n_sroot * sizeof(SRoot), st));
            scap = nc2;
        }
        if (hc.n_lleaf + 2 * (size_t)n > lcap) {
            size_t nc2 = std::max(lcap * 2, (size_t)hc.n_lleaf + 2 * n);
            GBCHK(llb.grow(nc2 * sizeof(LLeaf), (size_t)hc.n_lleaf * sizeof(LLeaf), st));
            lcap = nc2;
        }
        GBCHK(nc.ensure(4 * ((size_t)n + 1)));
        GBCHK(c0.ensure(4 * ((size_t)n + 1)));
        hipLaunchKernelGGL(k_nchunks, dim3(blocks(n + 1, 256)), dim3(256), 0, st, gn.as<GNode>(), lb, n,
                           nc.as<uint32_t>());
        size_t tbytes = tmp.bytes;
        GBCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tbytes, nc.as<uint32_t>(), c0.as<uint32_t>(), (int)n + 1, st));
        uint32_t nch = 0;
        GBCHK(hipMemcpyAsync(&nch, c0.as<uint32_t>() + n, 4, hipMemcpyDeviceToHost, st));
        GBCHK(hipStreamSynchronize(st));
        GBCHK(chunk_node.ensure(4 * (size_t)nch));
        GBCHK(part.ensure(4 * (size_t)BW * nch));
        GBCHK(cnt.ensure(8 * ((size_t)nch + 1)));
        GBCHK(off.ensure(8 * ((size_t)nch + 1)));
        hipLaunchKernelGGL(k_chunk_list, dim3(n), dim3(256), 0, st, gn.as<GNode>(), lb, c0.as<uint32_t>(),
                           chunk_node.as<uint32_t>());
        hipLaunchKernelGGL(k_bin, dim3(nch), dim3(256), 0, st, rec.as<float4>(), gn.as<GNode>(),
                           chunk_node.as<uint32_t>(), part.as<uint32_t>());
        hipLaunchKernelGGL(k_pick, dim3(n), dim3(PICK_GROUPS * BW), 0, st, gn.as<GNode>(), lb, part.as<uint32_t>(), (uint32_t)gcap,
                           srb.as<SRoot>(), (uint32_t)scap, llb.as<LLeaf>(), (uint32_t)lcap,
                           leafstart.as<uint32_t>(), ctr.as<Ctr>());
        hipLaunchKernelGGL(k_classify, dim3(nch), dim3(256), 0, st, rec.as<float4>(), gn.as<GNode>(),
                           chunk_node.as<uint32_t>(), cnt.as<uint64_t>());
        tbytes = tmp.bytes;
        GBCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tbytes, cnt.as<uint64_t>(), off.as<uint64_t>(), (int)nch + 1, st));
        hipLaunchKernelGGL(k_swap_write, dim3(nch), dim3(256), 0, st, rec.as<float4>(), gn.as<GNode>(),
                           chunk_node.as<uint32_t>(), off.as<uint64_t>(), SL.as<float4>(), SR.as<float4>(),
                           PL.as<uint32_t>(), PR.as<uint32_t>());
        hipLaunchKernelGGL(k_swap_apply, dim3(nch), dim3(256), 0, st, rec.as<float4>(), gn.as<GNode>(),
                           chunk_node.as<uint32_t>(), off.as<uint64_t>(), SL.as<float4>(), SR.as<float4>(),
                           PL.as<uint32_t>(), PR.as<uint32_t>());
        GBCHK(hipGetLastError());
        GBCHK(hipMemcpyAsync(&hc, ctr.p, sizeof(hc), hipMemcpyDeviceToHost, st));
        GBCHK(hipStreamSynchronize(st));
        if (hc.error) return "device BVH build failed (code " + std::to_string(hc.error) + ")";
        lb = le;
        le = hc.n_gnode;
    }
    // small subtrees
    Buf T;
    GBCHK(T.ensure(2 * (size_t)N * sizeof(BuildNode)));
    Buf fst, nxt;
    if (hc.n_sroot) {
        int dev = 0, n_cu = 256;
        GBCHK(hipGetDevice(&dev));
        GBCHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
        const uint32_t grid = std::min<uint32_t>(hc.n_sroot, (uint32_t)n_cu * 12u);
        GBCHK(fst.ensure((size_t)grid * SUB_STACK * sizeof(Frame)));
        GBCHK(nxt.ensure(4));
        GBCHK(hipMemsetAsync(nxt.p, 0, 4, st));
        hipLaunchKernelGGL(k_subtree, dim3(grid), dim3(64), 0, st, rec.as<float4>(), bnd, srb.as<SRoot>(), hc.n_sroot,
                           nxt.as<uint32_t>(), T.as<BuildNode>(), leafstart.as<uint32_t>(), ctr.as<Ctr>(),
                           fst.as<Frame>());
    }
    GBCHK(hipGetLastError());
    // leaf starts -> P (exclusive), P[N] = leaves
    GBCHK(t.P.ensure(4 * ((size_t)N + 1)));
    size_t tbytes = tmp.bytes;
    GBCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tbytes, leafstart.as<uint32_t>(), t.P.as<uint32_t>(), (int)N + 1,
                                           st));
    uint32_t n_leaves = 0;
    GBCHK(hipMemcpyAsync(&n_leaves, t.P.as<uint32_t>() + N, 4, hipMemcpyDeviceToHost, st));
    GBCHK(hipMemcpyAsync(&hc, ctr.p, sizeof(hc), hipMemcpyDeviceToHost, st));
    GBCHK(hipStreamSynchronize(st));
    if (hc.error) return "device BVH build failed (code " + std::to_string(hc.error) + ")";
    const size_t n_nodes = 2 * (size_t)n_leaves - 1;
    GBCHK(t.nodes.ensure(n_nodes * sizeof(BuildNode)));
    BuildNode* fin = t.nodes.as<BuildNode>();
    const uint32_t* P = t.P.as<uint32_t>();
    if (hc.n_sroot)
        hipLaunchKernelGGL(k_copy_subtrees, dim3(blocks(hc.n_sroot, 256)), dim3(256), 0, st, srb.as<SRoot>(),
                           hc.n_sroot, T.as<BuildNode>(), P, fin);
    if (hc.n_lleaf)
        hipLaunchKernelGGL(k_level_leaves, dim3(blocks(hc.n_lleaf, 256)), dim3(256), 0, st, llb.as<LLeaf>(),
                           hc.n_lleaf, rec.as<float4>(), bnd, P, fin);
    for (size_t l = levels.size(); l-- > 0;)
        hipLaunchKernelGGL(k_level_interior, dim3(blocks(levels[l].second, 256)), dim3(256), 0, st, gn.as<GNode>(),
                           levels[l].first, levels[l].second, P, fin);
    GBCHK(t.ids.ensure(4 * (size_t)N));
    hipLaunchKernelGGL(k_ids, dim3(blocks(N, 256)), dim3(256), 0, st, rec.as<float4>(), N, t.ids.as<uint32_t>());
    GBCHK(hipGetLastError());
    GBCHK(hipEventRecord(ev1, st));
    GBCHK(hipEventSynchronize(ev1));
    float ms = 0.0f;
    GBCHK(hipEventElapsedTime(&ms, ev0, ev1));
    (void)hipEventDestroy(ev0);
    (void)hipEventDestroy(ev1);
    if (kernel_ms) *kernel_ms = ms;
    t.n_nodes = (uint32_t)n_nodes;
    t.n_leaves = n_leaves;
    hs.depth = hc.max_depth;
    hs.max_leaf = hc.max_leaf;
    (void)t0;
    return std::string();
}

std::string download_tree(const DeviceTree& t, HostScene& hs, hipStream_t st) {
    hs.nodes.resize(t.n_nodes);
    hs.ids.resize(hs.n_obj);
    GBCHK(hipMemcpyAsync(hs.nodes.data(), t.nodes.p, (size_t)t.n_nodes * sizeof(BuildNode), hipMemcpyDeviceToHost, st));
    GBCHK(hipMemcpyAsync(hs.ids.data(), t.ids.p, 4 * (size_t)hs.n_obj, hipMemcpyDeviceToHost, st));
    GBCHK(hipStreamSynchronize(st));
    return std::string();
}

// ---- make_device_layout on the device (scene.cpp) -------------------------------
namespace gb {

// h[i] = interior node i with at least one interior child: it opens a record pair.
__global__ void k_lay_flags(const BuildNode* fin, uint32_t n, uint32_t* h) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    uint32_t v = 0;
    if (i < n) {
        const BuildNode nd = fin[i];
        if (nd.count == 0) v = (fin[nd.left].count == 0 || fin[nd.right].count == 0) ? 1u : 0u;
    }
    h[i] = v;
}

// The host pops interior nodes in preorder and gives the interior children of
// the k-th pair-opening node the records (2 + 2k, 2 + 2k + 1).
__global__ void k_lay_recof(const BuildNode* fin, uint32_t n, const uint32_t* H, int32_t* rec_of) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const BuildNode nd = fin[i];
    if (i == 0) rec_of[0] = nd.count == 0 ? 0 : -1;
    if (nd.count != 0) return;
    const bool li = fin[nd.left].count == 0, ri = fin[nd.right].count == 0;
    const int32_t base = (int32_t)(2u + 2u * H[i]);
    if (li) rec_of[nd.left] = base;
    if (ri) rec_of[nd.right] = li ? base + 1 : base;
}

// leaves in preorder = leaves by first; ordinal = P[first]
__global__ void k_lay_leaves(const BuildNode* fin, uint32_t n, const uint32_t* P, uint32_t* lfirst, uint2* lfun) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const BuildNode nd = fin[i];
    if (nd.count == 0) return;
    const uint32_t l = P[nd.first], c = (uint32_t)nd.count;
    lfirst[l] = (uint32_t)nd.first;
    // slot advance as a function of the running slot count's parity:
    // a leaf of >= 2 candidates starts at an even slot
    lfun[l] = c >= 2 ? make_uint2(c, c + 1) : make_uint2(c, c);
}

struct ParityCompose {  // (f then g) for the parity-dependent slot advance
    __host__ __device__ uint2 operator()(const uint2& f, const uint2& g) const {
        return make_uint2(f.x + ((f.x & 1u) ? g.y : g.x), f.y + (((1u + f.y) & 1u) ? g.y : g.x));
    }
};

__global__ void k_lay_slot0(const uint2* lfun, const uint2* scanned, uint32_t nl, uint32_t* slot0) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= nl) return;
    const uint32_t ns = scanned[l].x;  // slots before this leaf, from an even start
    const bool two = lfun[l].y != lfun[l].x;
    slot0[l] = ns + ((two && (ns & 1u)) ? 1u : 0u);
}

__device__ __forceinline__ void child_ref(const BuildNode* fin, int32_t c, const int32_t* rec_of, const uint32_t* P,
                                          const uint32_t* slot0, int32_t& ref, int32_t& cnt) {
    const BuildNode nd = fin[c];
    if (nd.count > 0) {
        const uint32_t ce = (uint32_t)nd.count < LEAF_CNT_ESC ? (uint32_t)nd.count : LEAF_CNT_ESC;
        ref = (int32_t)(LEAF_BIT | (ce << 24) | slot0[P[nd.first]]);
        cnt = nd.count;
    } else {
        ref = rec_of[c];
        cnt = 0;
    }
}

__global__ void k_lay_nodes(const BuildNode* fin, uint32_t n, const int32_t* rec_of, const uint32_t* P,
                            const uint32_t* slot0, DevNode* dn) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const BuildNode nd = fin[i];
    if (nd.count != 0) return;
    const BuildNode L = fin[nd.left], R = fin[nd.right];
    DevNode d;
    d.a[0] = L.mn.x; d.a[1] = L.mn.y; d.a[2] = L.mn.z; d.a[3] = L.mx.x;
    d.b[0] = L.mx.y; d.b[1] = L.mx.z; d.b[2] = R.mn.x; d.b[3] = R.mn.y;
    d.c[0] = R.mn.z; d.c[1] = R.mx.x; d.c[2] = R.mx.y; d.c[3] = R.mx.z;
    child_ref(fin, nd.left, rec_of, P, slot0, d.ref[0], d.cnt[0]);
    child_ref(fin, nd.right, rec_of, P, slot0, d.ref[1], d.cnt[1]);
    dn[rec_of[i]] = d;
}

// slot records: position p of the leaf order -> slot slot0[leaf] + (p - leaf.first)
__global__ void k_lay_slots(const uint32_t* ids, uint32_t N, const uint32_t* P, const uint32_t* lfirst,
                            const uint32_t* slot0, const uint2* lfun, const float4* rec_obj, const Aux* aux_obj,
                            float4* prims, Aux* aux) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    const uint32_t l = P[p + 1] - 1u, k = p - lfirst[l], s = slot0[l] + k, o = ids[p];
    const float4* src = rec_obj + 4 * (size_t)o;
    float4* dst = prims + 4 * (size_t)s;
    dst[0] = src[0];
    dst[1] = src[1];
    dst[2] = src[2];
    dst[3] = src[3];
    Aux a = aux_obj[o];
    if (k == 0) a.flags |= lfun[l].x << 8;  // candidate count of the leaf starting here
    aux[s] = a;
}

}  // namespace gb

std::string device_layout(const DeviceObjects& o, DeviceTree& t, hipStream_t st, DevMem& dnodes, DevMem& prims,
                          DevMem& aux, DeviceLayout& out, double* kernel_ms) {
    using namespace gb;
    const uint32_t N = o.n_obj, n = t.n_nodes, nl = t.n_leaves;
    const BuildNode* fin = t.nodes.as<BuildNode>();
    const uint32_t* P = t.P.as<uint32_t>();
    Buf h, H, rec_of, lfirst, lfun, lscan, slot0, tmp;
    hipEvent_t ev0, ev1;
    GBCHK(hipEventCreate(&ev0));
    GBCHK(hipEventCreate(&ev1));
    GBCHK(hipEventRecord(ev0, st));
    GBCHK(h.ensure(4 * ((size_t)n + 1)));
    GBCHK(H.ensure(4 * ((size_t)n + 1)));
    GBCHK(rec_of.ensure(4 * (size_t)n));
    GBCHK(lfirst.ensure(4 * (size_t)nl));
    GBCHK(lfun.ensure(8 * ((size_t)nl + 1)));
    GBCHK(lscan.ensure(8 * ((size_t)nl + 1)));
    GBCHK(slot0.ensure(4 * (size_t)nl));
    size_t tb1 = 0, tb2 = 0;
    GBCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb1, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)n + 1, st));
    GBCHK(hipcub::DeviceScan::ExclusiveScan(nullptr, tb2, (uint2*)nullptr, (uint2*)nullptr, ParityCompose(),
                                            make_uint2(0u, 0u), (int)nl + 1, st));
    GBCHK(tmp.ensure(std::max(tb1, tb2)));
    hipLaunchKernelGGL(k_lay_flags, dim3(blocks(n + 1, 256)), dim3(256), 0, st, fin, n, h.as<uint32_t>());
    size_t tb = tmp.bytes;
    GBCHK(hipcub::DeviceScan::ExclusiveSum(tmp.p, tb, h.as<uint32_t>(), H.as<uint32_t>(), (int)n + 1, st));
    hipLaunchKernelGGL(k_lay_recof, dim3(blocks(n, 256)), dim3(256), 0, st, fin, n, H.as<uint32_t>(),
                       rec_of.as<int32_t>());
    const uint2 ident = make_uint2(0u, 0u);
    GBCHK(hipMemcpyAsync(lfun.as<uint2>() + nl, &ident, 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_lay_leaves, dim3(blocks(n, 256)), dim3(256), 0, st, fin, n, P, lfirst.as<uint32_t>(),
                       lfun.as<uint2>());
    tb = tmp.bytes;
    GBCHK(hipcub::DeviceScan::ExclusiveScan(tmp.p, tb, lfun.as<uint2>(), lscan.as<uint2>(), ParityCompose(), ident,
                                            (int)nl + 1, st));
    hipLaunchKernelGGL(k_lay_slot0, dim3(blocks(nl, 256)), dim3(256), 0, st, lfun.as<uint2>(), lscan.as<uint2>(), nl,
                       slot0.as<uint32_t>());
    GBCHK(hipGetLastError());
    uint32_t Htot = 0;
    uint2 stot{0, 0};
    BuildNode root{};
    GBCHK(hipMemcpyAsync(&Htot, H.as<uint32_t>() + n, 4, hipMemcpyDeviceToHost, st));
    GBCHK(hipMemcpyAsync(&stot, lscan.as<uint2>() + nl, 8, hipMemcpyDeviceToHost, st));
    GBCHK(hipMemcpyAsync(&root, fin, sizeof(BuildNode), hipMemcpyDeviceToHost, st));
    GBCHK(hipStreamSynchronize(st));
    const bool root_interior = root.count == 0;
    out.n_dnodes = root_interior ? 2u + 2u * Htot : 0u;
    out.n_slots = stot.x;
    GBCHK(dnodes.ensure(sizeof(DevNode) * (size_t)std::max(out.n_dnodes, 1u)));
    GBCHK(prims.ensure(64 * (size_t)out.n_slots));
    GBCHK(aux.ensure(sizeof(Aux) * (size_t)out.n_slots));
    GBCHK(hipMemsetAsync(dnodes.p, 0, sizeof(DevNode) * (size_t)std::max(out.n_dnodes, 1u), st));
    GBCHK(hipMemsetAsync(prims.p, 0, 64 * (size_t)out.n_slots, st));
    GBCHK(hipMemsetAsync(aux.p, 0, sizeof(Aux) * (size_t)out.n_slots, st));
    hipLaunchKernelGGL(k_lay_nodes, dim3(blocks(n, 256)), dim3(256), 0, st, fin, n, rec_of.as<int32_t>(), P,
                       slot0.as<uint32_t>(), dnodes.as<DevNode>());
    hipLaunchKernelGGL(k_lay_slots, dim3(blocks(N, 256)), dim3(256), 0, st, t.ids.as<uint32_t>(), N, P,
                       lfirst.as<uint32_t>(), slot0.as<uint32_t>(), lfun.as<uint2>(), o.rec.as<float4>(),
                       o.aux.as<Aux>(), prims.as<float4>(), aux.as<Aux>());
    GBCHK(hipGetLastError());
    GBCHK(hipEventRecord(ev1, st));
    // root reference (make_device_layout: child_ref(0, ...))
    if (root_interior) {
        out.root_ref = 0;
        out.root_cnt = 0;
    } else {
        uint32_t s0 = 0;
        GBCHK(hipMemcpyAsync(&s0, slot0.p, 4, hipMemcpyDeviceToHost, st));
        GBCHK(hipStreamSynchronize(st));
        const uint32_t ce = (uint32_t)root.count < LEAF_CNT_ESC ? (uint32_t)root.count : LEAF_CNT_ESC;
        out.root_ref = (int32_t)(LEAF_BIT | (ce << 24) | s0);
        out.root_cnt = root.count;
    }
    const float rb[6] = {root.mn.x, root.mn.y, root.mn.z, root.mx.x, root.mx.y, root.mx.z};
    memcpy(out.root_box, rb, sizeof(rb));
    GBCHK(hipStreamSynchronize(st));
    float ms = 0.0f;
    GBCHK(hipEventElapsedTime(&ms, ev0, ev1));
    (void)hipEventDestroy(ev0);
    (void)hipEventDestroy(ev1);
    if (kernel_ms) *kernel_ms = ms;
    return std::string();
}

}  // namespace khp

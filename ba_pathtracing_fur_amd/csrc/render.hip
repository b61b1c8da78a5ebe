// render.hip -- the MI355X wavefront integrator and the C-ABI (include/kirk_hip.h).
//
// One khp_render call replaces KIRK's PathTracer::render/processSegment/
// traceRays (CPU_PathTracer.cpp:17-209).  Instead of KIRK's per-pixel AoS
// loop with a fork-join per bounce, the paths of a whole batch (owned pixels x
// samples) live in SoA buffers in HBM and each bounce runs three kernels:
//   extend  : persistent, wave-fetched closest-hit BVH2 traversal
//   shade   : light hit test, environment/light/material shaders, BSDF sample,
//             NEE shadow-ray setup; wave ballot compaction of the next ray
//             queue and of the shadow queue
//   shadow  : persistent any-hit traversal, then the deferred colour add
// followed by one accumulate kernel per batch (KIRK's running mean).  All
// counts stay on the device, so a frame is enqueued without host syncs.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <string>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>
#include <type_traits>
#include <vector>

#include "device.h"
#include "device_build.h"
#include "lightpath.h"

using namespace khp;

// ============================================================================
//  wavefront state
// ============================================================================
#ifndef KHP_MAX_SEG
#define KHP_MAX_SEG 64
#endif
struct alignas(128) Counters {
    uint32_t nq[2];        // ray queue sizes: front part (predicted long rays)
    uint32_t nqb[2];       // back part (predicted short rays), stored from the end of the buffers
    uint32_t pad_a[28];
    uint32_t fetch_ext[KHP_MAX_SEG * 32];  // queue-segment claim cursors, one 128-B line each
    unsigned long long ext_rays, sh_rays;
    unsigned long long node_visits, prim_tests, sh_node_visits, sh_prim_tests, spills;
    unsigned long long pruned, sh_pruned;  // entries popped only to fail the prune test
    unsigned long long iters, lanes_busy, sh_iters, sh_lanes_busy;  // wave iterations, lanes with work
    unsigned long long step_cycles[4];  // diagnostic builds only (KHP_PATH_PROFILE), else 0
};

// One bounce's shadow-ray queue (count + claim cursors).  Two of them
// (bounce parity) let k_shade of bounce b+1 fill one while k_shadow of bounce
// b drains the other on the second stream.
struct alignas(128) ShadowQ {
    uint32_t nsh;          // front part (predicted long shadow rays)
    uint32_t nshb;         // back part
    uint32_t pad[30];
    uint32_t fetch[KHP_MAX_SEG * 32];
};

#ifndef KHP_MAX_FUSE
#define KHP_MAX_FUSE 32
#endif
struct Wave {
    float* qo[2][3];
    float* qd[2][3];
    uint32_t* qpid[2];
    float* ht;
    int32_t* hslot;
    // Per-path state, one 16-B record per array so that k_shade and
    // k_shadow_finish, which reach paths in queue order (scattered pids after
    // bounce 0), touch one line per array instead of one per component:
    float4* TFq[2];      // per queue slot (moves with the path's ray): throughput T.xyz, BSDF flags (bits) in w
    float4* CKq[2];      // per queue slot: colour C.xyz, RNG key (bits) in w
    float4* CK;          // per path: the final colour, written when the path ends (k_accumulate reads it)
    uint8_t* vis;        // shadow-ray occlusion flag per shadow record (this parity)
    ShadowQ* shq;        // shadow queue of this parity
    float4* sh;          // shs float4 per shadow record
    // float4 per shadow record: 4 for the next-event records of k_shade (o + t_max,
    // d + state destination, the colour add if unoccluded, the add if occluded), 6 for
    // the light-path variant's connection records and the batch ray queries
    uint32_t shs;
    Counters* cnt;
    const uint32_t* pix;  // owned pixel ids (y*W+x)
    uint32_t P;           // pixels in this chunk
    uint32_t p_off;       // chunk offset into pix
    uint32_t W, H;
    uint32_t seed;
    uint32_t sample0;     // global sample index of chunk sample 0
    uint32_t n_samples;   // samples in this chunk (per frame)
    uint32_t n_frames;    // fused frames in this chunk
    uint32_t pix_major;   // path numbering (khp_ctx_params.path_order): 0 frame-major, else pixel-major
    uint8_t* pixheavy;    // path_order 2: per image pixel, its last camera ray took > heavy_T iterations (null: off)
    uint32_t cam0;        // bounce 0 computes camera rays in place (no k_generate queue)
    uint32_t q_cur, q_bounce;   // k_path from the queue (hybrid batches): the queue's parity and bounce
    uint32_t fsample0[KHP_MAX_FUSE];  // per fused frame: global sample index of chunk sample 0
    uint32_t depth;
    uint8_t* heavy;       // per queue slot: the ray's traversal took more than heavy_T iterations
    uint32_t cap;         // queue / path capacity of this set
    uint32_t heavy_T;
    // shade_order 1 (hit sorting): k_shade takes queue slot perm[iv] instead of q_phys(iv)
    uint32_t* perm;       // null: queue order
    uint8_t* hkey;        // shading class of queue entry iv (k_hit_class -> k_hit_scatter)
    uint32_t* hcls;       // [0,16): entries per class, [16,32): scatter cursors per class
    BdptDev bd;           // light-path variant (ABI 7); bd.on = 0: next-event estimate
    // Ray sorting (khp_ctx_params.sort_from): this bounce's queue was regrouped by
    // origin cell; qo/qd/qpid of the current parity then point at the regrouped
    // columns and qsrc[slot] is the slot that holds the entry's path state (TFq,
    // CKq), which stays where k_shade and the shadow finish left it.  Null: identity.
    const uint32_t* qsrc;
};

// Path numbering of a chunk.  Frame-major: path = (frame * P + pixel) * n_samples
// + sample.  Pixel-major: path = (pixel * n_frames + frame) * n_samples + sample,
// so every fused frame's samples of one pixel are adjacent.  Paths are
// independent and each pixel's samples are summed in (frame, sample) order either
// way, so the numbering changes no result.
__device__ __forceinline__ void path_coords(const Wave& Wv, uint32_t pid, uint32_t& fr, uint32_t& p_local,
                                            uint32_t& s_local) {
    if (Wv.pix_major) {
        const uint32_t per_pix = Wv.n_frames * Wv.n_samples;
        p_local = pid / per_pix;
        const uint32_t r = pid - p_local * per_pix;
        fr = r / Wv.n_samples;
        s_local = r - fr * Wv.n_samples;
    } else {
        const uint32_t per_frame = Wv.P * Wv.n_samples;
        fr = pid / per_frame;
        const uint32_t pf = pid - fr * per_frame;
        p_local = pf / Wv.n_samples;
        s_local = pf - p_local * Wv.n_samples;
    }
}

__device__ __forceinline__ size_t path_index(const Wave& Wv, uint32_t fr, uint32_t p_local, uint32_t s_local) {
    return Wv.pix_major ? ((size_t)p_local * Wv.n_frames + fr) * Wv.n_samples + s_local
                        : ((size_t)fr * Wv.P + p_local) * Wv.n_samples + s_local;
}



// Longest-first queues.  A persistent traversal launch ends when its slowest
// ray does; if long rays are claimed last, each launch ends one long-ray
// latency (~1 ms inside the hairball) after its queue has drained.  k_shade
// therefore writes the next bounce's rays (and the shadow rays) of paths
// whose last traversal was long to the front of the queue buffers and the
// others to the back (stored from the end), and the claim order takes the
// front part of every claim segment first.  Paths are independent, so the
// order changes no result.
__device__ __forceinline__ uint32_t q_phys(uint32_t v, uint32_t nf, uint32_t cap) {
    return v < nf ? v : cap - 1u - (v - nf);
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }

// wave-level stream compaction: one atomic per wave, order-preserving in the wave.
__device__ __forceinline__ uint32_t wave_alloc(bool pred, uint32_t* counter) {
    unsigned long long mask = __ballot(pred);
    uint32_t lane = lane_id();
    uint32_t prefix = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
    uint32_t base = 0;
    if (lane == 0 && mask) base = atomicAdd(counter, (uint32_t)__popcll(mask));
    base = __shfl(base, 0);
    return base + prefix;
}

// Wave-level allocation of cnt (< 32) consecutive entries per lane, callable
// from divergent code: the prefix sum is built from one ballot per bit of
// cnt, so lanes that do not execute the call count nothing.
__device__ __forceinline__ uint32_t wave_alloc_n(uint32_t cnt, uint32_t* counter) {
    const uint32_t lane = lane_id();
    const unsigned long long lt = (1ull << lane) - 1ull;
    uint32_t prefix = 0, total = 0;
    for (int bit = 0; bit < 5; ++bit) {
        const unsigned long long m = __ballot((cnt >> bit) & 1u);
        prefix += (uint32_t)__popcll(m & lt) << bit;
        total += (uint32_t)__popcll(m) << bit;
    }
    const uint32_t leader = (uint32_t)__ffsll((long long)__ballot(1)) - 1u;
    uint32_t base = 0;
    if (lane == leader && total) base = atomicAdd(counter, total);
    base = __shfl(base, (int)leader);
    return base + prefix;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// ---- generate: camera rays (PathTracer::generatePrimaryRays, CPU_PathTracer.cpp:118-127;
//      Camera::getRayFromPixel, Camera.cpp:59-66) -------------------------------------------
// Camera ray and RNG key of path pid.  k_generate writes them to the bounce-0
// queue; with Wave::cam0 set, k_extend and k_shade compute them in place at
// bounce 0 instead (queue slot = path there), the same operations.
__device__ __forceinline__ Ray camera_path(const DevScene& S, const Wave& Wv, uint32_t pid, uint32_t& key,
                                           uint32_t s_off = 0u) {
    // the samples of one pixel are adjacent paths (path_coords), so a wave traces
    // a few neighbouring pixels x all their samples (cache reuse); s_off: the
    // render-ahead set's sample offset (k_path)
    uint32_t fr, p_local, s_local;
    path_coords(Wv, pid, fr, p_local, s_local);
    const uint32_t pixel = Wv.pix[Wv.p_off + p_local];
    const uint32_t x = pixel % Wv.W, y = pixel / Wv.W;
    key = path_key(Wv.seed, pixel, Wv.fsample0[fr] + s_local + s_off);
    const float u1 = draw_u01(key, dim_of(0, P_CAM_X)), u2 = draw_u01(key, dim_of(0, P_CAM_Y));
    const khp_camera& cam = S.cam;
    const float s1 = ((float)x + u1) * cam.pixel_size, s2 = ((float)y + u2) * cam.pixel_size;
    const v3 dir = ((ld3(cam.bottom_left) + ld3(cam.axis_x) * s1) + ld3(cam.axis_y) * s2) - ld3(cam.position);
    return make_ray(ld3(cam.position), dir);
}

__global__ __launch_bounds__(256) void k_generate(DevScene S, Wave Wv) {
    uint32_t n = Wv.P * Wv.n_samples * Wv.n_frames;
    uint32_t pid = blockIdx.x * blockDim.x + threadIdx.x;
    if (pid == 0) {
        Wv.cnt->nq[0] = n;   // primary rays: all in the front part
        Wv.cnt->nqb[0] = 0;
    }
    if (pid >= n) return;
    uint32_t key;
    const Ray r = camera_path(S, Wv, pid, key);
    Wv.qo[0][0][pid] = r.o.x; Wv.qo[0][1][pid] = r.o.y; Wv.qo[0][2][pid] = r.o.z;
    Wv.qd[0][0][pid] = r.d.x; Wv.qd[0][1][pid] = r.d.y; Wv.qd[0][2][pid] = r.d.z;
    Wv.qpid[0][pid] = pid;
    Wv.TFq[0][pid] = make_float4(1.0f, 1.0f, 1.0f, f_from_bits(0u));  // queue slot = path at bounce 0
    Wv.CKq[0][pid] = make_float4(0.0f, 0.0f, 0.0f, f_from_bits(key));
}

// Wave::cam0: the bounce-0 queue is implicit (every path, in path order).
__global__ void k_start(Counters* c, uint32_t n) {
    c->nq[0] = n;
    c->nqb[0] = 0;
}

__global__ void k_prep(Counters* c, ShadowQ* q, int cur) {
    int nxt = cur ^ 1;
    c->nq[nxt] = 0;
    c->nqb[nxt] = 0;
    q->nsh = 0;
    q->nshb = 0;
    for (int g = 0; g < KHP_MAX_SEG; ++g) {
        c->fetch_ext[32 * g] = 0;
        q->fetch[32 * g] = 0;
    }
    c->ext_rays += c->nq[cur] + c->nqb[cur];
}

// ---- persistent lane-refill traversal -------------------------------------------------------
// Every lane owns one ray at a time.  When at least REFILL lanes of a wave are
// idle, the wave claims that many new rays with a single atomic and the idle
// lanes start them, so a wave never waits for its slowest ray to admit new
// work (Aila & Laine's persistent "while-while" with speculative refill).
// Measured on the metric row: 8-entry LDS rings, refill at 24
// idle lanes and 6 waves per SIMD (72 VGPRs, 6 x 24 KB of LDS rings per CU)
// are the best of the variants tried.
#ifndef KHP_EXT_RING
#define KHP_EXT_RING 8
#endif
#ifndef KHP_EXT_WAVES
#define KHP_EXT_WAVES 6
#endif
#ifndef KHP_EXT_REFILL
#define KHP_EXT_REFILL 24
#endif
#ifndef KHP_SH_RING
#define KHP_SH_RING 8
#endif
#ifndef KHP_SH_WAVES
#define KHP_SH_WAVES 6
#endif
constexpr int RING = KHP_SH_RING;         // LDS ring entries per lane (3 x 4 B each), k_shadow
constexpr int REFILL = 24;                // refill when >= REFILL lanes are idle
constexpr int TRAV_WAVES = KHP_SH_WAVES;  // __launch_bounds__ waves per SIMD, k_shadow
constexpr int EXT_RING = KHP_EXT_RING;    // the same for k_extend
constexpr int EXT_WAVES = KHP_EXT_WAVES;
#ifndef KHP_EXT_WAVES_W
#define KHP_EXT_WAVES_W 6
#endif
constexpr int EXT_WAVES_W = KHP_EXT_WAVES_W;  // k_extend over the two-level records (80 VGPRs: 6 waves)
// k_extend's refill threshold per instance (bounce 0 / 64-B loop / two-level
// loop), default KHP_EXT_REFILL for each; 16 and 32 measured for each
#ifndef KHP_REFILL_CAM   // 28 in round 5 (bounce 0: 4.56 against 4.72 ms per frame, +0.5%)
#define KHP_REFILL_CAM 28
#endif
#ifndef KHP_REFILL_NARROW   // 28 in round 5 (bounce 1: 7.17 against 7.21-7.25 ms per frame, +0.2%)
#define KHP_REFILL_NARROW 28
#endif
#ifndef KHP_REFILL_WIDE   // 16 since the ray regrouping (round 5: lane use 0.73 -> 0.76 at bounce 2, +0.3%)
#define KHP_REFILL_WIDE 16
#endif
constexpr size_t LDS_BYTES = 3 * RING * TRAV_BLOCK * sizeof(uint32_t);
constexpr size_t EXT_LDS_BYTES = 3 * EXT_RING * TRAV_BLOCK * sizeof(uint32_t);
// Bounce 0 (camera rays computed in place, k_extend<., true, .>): cache-served and
// latency-bound, so the 64-B loop (59 VGPRs) runs 8 waves per SIMD there, with
// 6-entry rings so 32 one-wave blocks fit a CU's LDS.
#ifndef KHP_CAM_RING
#define KHP_CAM_RING 6
#endif
#ifndef KHP_CAM_WAVES
#define KHP_CAM_WAVES 8
#endif
constexpr int CAM_RING = KHP_CAM_RING;
constexpr int CAM_WAVES = KHP_CAM_WAVES;
constexpr size_t CAM_LDS_BYTES = 3 * CAM_RING * TRAV_BLOCK * sizeof(uint32_t);
template <bool STATS, bool TOP = false>
using TravStack = LdsStack<RING, STATS, TOP>;
template <bool STATS, bool CAM = false, bool TOP = false>
using ExtStack = LdsStack<CAM ? CAM_RING : EXT_RING, STATS, TOP>;
constexpr size_t TOP_LDS_BYTES = TOP_NODES * sizeof(DevNode);   // added to a TOP instance's LDS

struct SpillArea {
    int4* base;
    uint32_t stride;   // lanes in the grid
};

// Work claiming with L2 affinity.  Blocks b and b+8 run on the same XCD
// (round-robin placement -- used for speed only, never for correctness), and
// each XCD has its own 4 MiB L2.  The queue is cut into NSEG contiguous
// segments; the waves of block group g = blockIdx.x % 8 drain segments
// [g*K, g*K + K) first, so each L2 serves one band of the frame (primary rays:
// a band of tiles; secondary and shadow rays: the matching region of the
// scene), then move on to the next segments so no XCD idles at the end of the
// launch.  K = 4 sub-segments per XCD spread the claim atomics over more lines.
constexpr uint32_t SEG_PER_XCD = 4;
constexpr uint32_t NSEG = 8u * SEG_PER_XCD;
static_assert(NSEG <= KHP_MAX_SEG, "claim cursors");
// Claim blocks (KHP_CLAIM_BLOCK_LOG2 = L > 0): instead of one contiguous slice
// per segment, the queue is cut into blocks of 2^L entries dealt round-robin to
// the NSEG segments (block b to segment b % NSEG), so all segments sweep the
// queue side by side and the rays in flight on the chip come from one window
// of NSEG x 2^L entries (with pixel-major paths: a compact patch of the image,
// so the XCDs share the Infinity Cache's subtrees).  L = 0: contiguous slices.
// Measured: 2^7..2^9 +0.9..1.3% over contiguous slices; 2^9 kept.
#ifndef KHP_CLAIM_BLOCK_LOG2
#define KHP_CLAIM_BLOCK_LOG2 9
#endif
// Two-level node records for k_extend (traverse.h iterw); 0: the 64-B loop only.
// KHP_WIDE_FROM: the default first bounce that uses them (khp_ctx_params.wide_from,
// ABI 10).  The camera and first secondary bounces are cache-served and
// issue-bound, where the two-level step (4 boxes per step, 80 VGPRs) loses;
// from bounce 2 line fetches bound the loop, and it takes a third fewer steps
// (DESIGN.md §4).
#ifndef KHP_WIDE
#define KHP_WIDE 1
#endif
#ifndef KHP_WIDE_FROM
#define KHP_WIDE_FROM 2   // default of khp_ctx_params.wide_from
#endif
// The shadow stage (any hit) of bounce b uses them from max(wide_from, this).
#ifndef KHP_WIDE_SH_FROM
#define KHP_WIDE_SH_FROM 2
#endif
constexpr uint32_t CB_LOG = KHP_CLAIM_BLOCK_LOG2;
constexpr uint32_t CB_MASK = (1u << CB_LOG) - 1u;
struct Claimer {
    uint32_t* fetch;  // NSEG cursors, one 128-B line each
    uint32_t nf, nl, cap;  // front / back parts, buffer capacity (longest-first queues)
    uint32_t sf, sl;  // claim blocks: entries of each part per segment (padded to whole blocks)
    uint32_t sg;      // segment this wave is draining (wave-uniform)
    uint32_t rseg;    // segment of the current reservation
    uint32_t tried;   // segments found exhausted
    uint32_t res_lo, res_hi;  // reserved, not yet handed out
    // Segment g holds its share of the front part followed by its share of the
    // back part: long rays first everywhere.  Contiguous slices (L = 0): the
    // slice [nf*g/NSEG, nf*(g+1)/NSEG) of each part.  Claim blocks (L > 0): each
    // part is padded to NSEG*K blocks of 2^L entries, and segment g takes blocks
    // g, g + NSEG, g + 2*NSEG, ...; entries in the padding are handed out as
    // empty (the lane stays idle) -- at most NSEG*2^L per part.
    __device__ __forceinline__ void init(uint32_t* f, uint32_t front, uint32_t back, uint32_t capacity) {
        fetch = f;
        nf = front;
        nl = back;
        cap = capacity;
        const uint32_t per = NSEG << CB_LOG;
        sf = CB_LOG ? ((front + per - 1u) / per) << CB_LOG : 0u;
        sl = CB_LOG ? ((back + per - 1u) / per) << CB_LOG : 0u;
        rseg = 0;
        sg = (blockIdx.x % 8u) * SEG_PER_XCD + (blockIdx.x / 8u) % SEG_PER_XCD;
        tried = 0;
        res_lo = res_hi = 0;
    }
    // The same claim geometry over another cursor array (render-ahead: the next set,
    // which has the same number of paths).
    __device__ __forceinline__ void retarget(uint32_t* f) {
        fetch = f;
        rseg = 0;
        sg = (blockIdx.x % 8u) * SEG_PER_XCD + (blockIdx.x / 8u) % SEG_PER_XCD;
        tried = 0;
        res_lo = res_hi = 0;
    }
    __device__ __forceinline__ uint32_t hlo(uint32_t g) const { return (uint32_t)((uint64_t)nf * g / NSEG); }
    __device__ __forceinline__ uint32_t llo(uint32_t g) const { return (uint32_t)((uint64_t)nl * g / NSEG); }
    __device__ __forceinline__ uint32_t lo(uint32_t g) const { return CB_LOG ? g * (sf + sl) : hlo(g) + llo(g); }
    // Physical queue slot of virtual index v of the current reservation; false
    // for an entry of the claim-block padding (no ray).
    __device__ __forceinline__ bool phys(uint32_t v, uint32_t& idx) const {
        const uint32_t local = v - lo(rseg);
        if (CB_LOG == 0) {
            const uint32_t hf = hlo(rseg + 1) - hlo(rseg);
            idx = local < hf ? hlo(rseg) + local : cap - 1u - (llo(rseg) + (local - hf));
            return true;
        }
        const bool front = local < sf;
        const uint32_t j = front ? local : local - sf;
        const uint32_t m = (((j >> CB_LOG) * NSEG + rseg) << CB_LOG) | (j & CB_MASK);
        idx = front ? m : cap - 1u - m;
        return m < (front ? nf : nl);
    }
    // Reserve up to `want` indices from the current segment (moving on when it runs dry).
    __device__ __forceinline__ void reserve(uint32_t want) {
        while (res_lo >= res_hi && tried < NSEG) {
            uint32_t base = 0;
            if (lane_id() == 0) base = atomicAdd(&fetch[32 * sg], want);
            base = __shfl(base, 0);
            const uint32_t s0 = lo(sg), len = lo(sg + 1) - s0;
            if (base < len) {
                res_lo = s0 + base;
                res_hi = s0 + (base + want < len ? base + want : len);
                rseg = sg;
            }
            if (base + want >= len) {
                sg = (sg + 1) % NSEG;
                ++tried;
            }
        }
    }
    // Hands indices to the idle lanes; returns true for this lane if it got one (my).
    // Sets done once every segment is drained and the reservoir is empty.
    __device__ __forceinline__ bool claim(unsigned long long idle, uint32_t& my, bool& done) {
        const uint32_t lane = lane_id();
        const uint32_t k = (uint32_t)__popcll(idle);
        reserve(k);
        const uint32_t avail = res_hi - res_lo, take = k < avail ? k : avail;
        const uint32_t off = (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
        my = res_lo + off;
        const bool got = (idle >> lane & 1ull) && off < take;
        res_lo += take;
        if (tried >= NSEG && res_lo >= res_hi) done = true;
        return got;
    }
};

// Adds one traversal kernel's instrumented counters to the wavefront counters.
template <class Stack>
__device__ __forceinline__ void flush_stats(const TravStats& st, const Stack& stk, unsigned long long wit,
                                            unsigned long long wbusy, unsigned long long* nodes,
                                            unsigned long long* prims, unsigned long long* pruned,
                                            unsigned long long* iters, unsigned long long* busy,
                                            unsigned long long* spills) {
    const unsigned long long a = wave_sum((unsigned long long)st.nodes), b = wave_sum((unsigned long long)st.prims);
    const unsigned long long pr = wave_sum((unsigned long long)st.pruned);
    const unsigned long long sp = wave_sum((unsigned long long)stk.spills);
    if (lane_id() == 0) {
        atomicAdd(nodes, a);
        atomicAdd(prims, b);
        atomicAdd(pruned, pr);
        atomicAdd(iters, wit);
        atomicAdd(busy, wbusy);
        atomicAdd(spills, sp);
    }
}

// path_order 2 (heavy-first pixels): the camera ray of path pid took more than
// heavy_T iterations.  The samples of a pixel race on its flag; any of their
// values is a valid hint (k_pix_order only reorders the pixel list).
__device__ __forceinline__ void mark_pixel(const Wave& Wv, uint32_t pid, bool long_ray) {
    uint32_t fr, p_local, s_local;
    path_coords(Wv, pid, fr, p_local, s_local);
    Wv.pixheavy[Wv.pix[Wv.p_off + p_local]] = long_ray ? 1 : 0;
}

// path_order 2: the batch's pixel list with the pixels whose last camera ray was
// long first (front part, ascending) and the others after them (back part,
// filled from the end).  A permutation of the owned pixels: paths are
// independent and each pixel's samples are summed in sample order, so the
// order changes no result; it moves the longest camera rays to the start of
// every bounce-0 launch instead of leaving them to its tail.
__global__ __launch_bounds__(256) void k_pix_order(const uint32_t* __restrict__ pix, uint32_t n,
                                                  const uint8_t* __restrict__ heavy, uint32_t* __restrict__ out,
                                                  uint32_t* cnt) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = i < n;
    const uint32_t px = in ? pix[i] : 0u;
    const bool hv = in && heavy[px] != 0;
    const uint32_t f = wave_alloc(hv, &cnt[0]);
    const uint32_t b = wave_alloc(in && !hv, &cnt[1]);
    if (hv) out[f] = px;
    else if (in) out[n - 1u - b] = px;
}

// ---- extend: closest hit for every queued ray ------------------------------------------
// CAM: bounce 0 with Wave::cam0 -- the ray of queue slot idx (= path idx) is
// the camera ray, computed here instead of loaded.
// WIDE: the two-level records (S.wide, traverse.h iterw) instead of the 64-B loop.
// TOP: the tree's top records staged in LDS (khp_ctx_params.lds_nodes; 64-B loop only).
template <bool STATS, bool CAM = false, bool WIDE = false, bool TOP = false>
__global__ __launch_bounds__(TRAV_BLOCK, WIDE ? EXT_WAVES_W : CAM ? CAM_WAVES : EXT_WAVES) void k_extend(DevScene S, Wave Wv, int cur, SpillArea spill) {
    extern __shared__ uint32_t lds[];
    const uint32_t nf = Wv.cnt->nq[cur], nb = Wv.cnt->nqb[cur];
    ExtStack<STATS, CAM, TOP> stk;
    stk.init(lds, spill.base, spill.stride);
    if (TOP) stk.stage_top(S.top);
    TravStats st{0, 0, 0};
    TravRay tr;
    Hit h;
    Cur c{0u, 0.0f, 0.0f, false};
    LeafCur lf{0u, 0u, 0.0f, 0.0f, 0.0f, 0.0f, -1};
    bool has = false, exhausted = false;
    uint32_t idx = 0, mode = 0u;
    unsigned long long wit = 0, wbusy = 0;  // STATS: wave iterations, busy lanes
    uint32_t it = 0;  // this lane's iterations on its current ray (longest-first queues)
    Claimer cl;
    cl.init(Wv.cnt->fetch_ext, nf, nb, Wv.cap);
    constexpr int refill = WIDE ? KHP_REFILL_WIDE : CAM ? KHP_REFILL_CAM : KHP_REFILL_NARROW;
    for (;;) {
        unsigned long long idle = __ballot(!has);
        if (!exhausted && __popcll(idle) >= refill) {
            uint32_t my;
            const bool got = cl.claim(idle, my, exhausted);
            if (!has && got && cl.phys(my, idx)) {
                it = 0;
                Ray r;
                if (CAM) {
                    uint32_t key_unused;
                    r = camera_path(S, Wv, idx, key_unused);
                } else {
                    r.o = mk(Wv.qo[cur][0][idx], Wv.qo[cur][1][idx], Wv.qo[cur][2][idx]);
                    r.d = mk(Wv.qd[cur][0][idx], Wv.qd[cur][1][idx], Wv.qd[cur][2][idx]);
                }
                trav_setup(tr, r);
                h.t = FLT_MAX_;
                h.slot = -1;
                h.u = h.v = 0.0f;
                lf.left = 0;
                has = (STATS || !ray_has_nan(r)) && trav2_begin<STATS>(S, tr, h.t, stk, mode, c, lf, st);
                if (!has) {  // missed the root box, or a NaN ray (no hit, see ray_has_nan)
                    Wv.ht[idx] = h.t;
                    Wv.hslot[idx] = -1;
                    Wv.heavy[idx] = 0;
                    if (CAM && Wv.pixheavy) mark_pixel(Wv, idx, false);
                }
            }
        }
        unsigned long long act = __ballot(has);
        if (act == 0) {
            if (exhausted) break;
            continue;
        }
        for (;;) {
            if (STATS) {
                unsigned long long wm = __ballot(has && (mode == M_NODE || mode == M_LEAF));
                ++wit;
                wbusy += (uint32_t)__popcll(wm);
            }
            if (has) {
                bool occ_unused;
                ++it;
                const bool fin = WIDE ? iterw<false, STATS>(S, tr, h, 0.0f, stk, mode, c, lf, st, occ_unused)
                                      : iter2<false, STATS>(S, tr, h, 0.0f, stk, mode, c, lf, st, occ_unused);
                if (fin) {
                    // the output addresses are formed here, not kept live through the loop
                    uint32_t j = idx;
                    asm volatile("" : "+v"(j));
                    Wv.ht[j] = h.t;
                    Wv.hslot[j] = h.slot;
                    Wv.heavy[j] = it > Wv.heavy_T ? 1 : 0;
                    if (CAM && Wv.pixheavy) mark_pixel(Wv, j, it > Wv.heavy_T);
                    has = false;
                }
            }
            act = __ballot(has);
            if (act == 0 || (!exhausted && 64 - __popcll(act) >= refill)) break;
        }
    }
    if (STATS)
        flush_stats(st, stk, wit, wbusy, &Wv.cnt->node_visits, &Wv.cnt->prim_tests, &Wv.cnt->pruned, &Wv.cnt->iters,
                    &Wv.cnt->lanes_busy, &Wv.cnt->spills);
}

// Host-side launch of the k_extend instance for (stats, camera rays in place, wide records).
static void launch_extend(bool stats, bool cam, bool wide, int grid, hipStream_t s, const DevScene& S, const Wave& W,
                          int cur, SpillArea sp, bool top = false) {
    const dim3 g(grid), b(TRAV_BLOCK);
    if (top && !stats && !wide && S.top) {   // the top records in LDS (lds_nodes)
        if (cam) hipLaunchKernelGGL((k_extend<false, true, false, true>), g, b, CAM_LDS_BYTES + TOP_LDS_BYTES, s, S, W, cur, sp);
        else hipLaunchKernelGGL((k_extend<false, false, false, true>), g, b, EXT_LDS_BYTES + TOP_LDS_BYTES, s, S, W, cur, sp);
        return;
    }
#define KHP_EXT(ST, CA, WI) \
    hipLaunchKernelGGL((k_extend<ST, CA, WI>), g, b, CA ? CAM_LDS_BYTES : EXT_LDS_BYTES, s, S, W, cur, sp)
    if (wide) {
        if (stats) { if (cam) KHP_EXT(true, true, true); else KHP_EXT(true, false, true); }
        else { if (cam) KHP_EXT(false, true, true); else KHP_EXT(false, false, true); }
    } else {
        if (stats) { if (cam) KHP_EXT(true, true, false); else KHP_EXT(true, false, false); }
        else { if (cam) KHP_EXT(false, true, false); else KHP_EXT(false, false, false); }
    }
#undef KHP_EXT
}

// ---- light-path variant (khp_bdpt_params, ABI 7; lightpath.h) ----------------------------
// The surface at a closest hit: normal, hair frame and material (k_shade's
// calcNormal / calcTcoord code; Cylinder.cpp:230-260, Triangle.cpp:244-254).
__device__ __forceinline__ void textured_material(const DevScene& S, const Aux& ax, const float4* pr, v3 loc,
                                               const ShadeCtx& s, float bu, float bv, khp_material& out);
template <bool TEX>
__device__ __forceinline__ v3 surface_at(const DevScene& S, const Ray& r, const Hit& h, ShadeCtx& s,
                                         khp_material& mres) {
    const Aux ax = S.aux[h.slot];
    const float4* pr = S.prims + 4 * (size_t)h.slot;
    s.m = &S.mats[ax.mat];
    v3 nrm;
    float bu = 0.0f, bv = 0.0f;  // barycentrics of a triangle hit (Hit::u, v are not used: tri_uv)
    if (ax.flags & 1u) {
        const float4 c0 = pr[0], c1 = pr[1], c2 = pr[2], c3 = pr[3];
        s.U = mk(c1.x, c1.y, c1.z);
        s.V = mk(c2.x, c2.y, c2.z);
        s.W = mk(c3.x, c3.y, c3.z);
        const v3 Q = follow(r, h.t);
        const float tt = dot(Q, s.V) - ax.base_d;
        const v3 q1 = Q - s.V * tt;
        const v3 nn = normalize(q1 - mk(c0.x, c0.y, c0.z));
        nrm = normalize(nn + s.V * c1.w);
    } else {
        tri_uv(pr[0], pr[1], pr[2], r, bu, bv);  // the hit's barycentrics (traversal keeps t and slot only)
        const float* tn = S.tri_nrm + 9 * (size_t)ax.obj;
        const float bx = (1.0f - bu) - bv;
        nrm = normalize((ld3(tn) * bx + ld3(tn + 3) * bu) + ld3(tn + 6) * bv);
        const float* tf = S.tri_frame + 9 * (size_t)ax.obj;
        s.U = ld3(tf);
        s.V = ld3(tf + 3);
        s.W = ld3(tf + 6);
    }
    s.n = nrm;
    if (TEX) {  // calcTcoord (traceRay, CPU_PathTracer.cpp:178-179), then the textured parameters
        mres = S.mats[ax.mat];
        textured_material(S, ax, pr, follow(r, h.t), s, bu, bv, mres);
        s.m = &mres;
    }
    return nrm;
}

// One light subpath per thread (lbb_construction.compute:195-403; the
// oracle's light_subpath): thread t = (sample slot q, subpath s, light) writes
// vertices [t*J, t*J + J) of bd.lv.  Sample slot q = frame * n_samples + sample.
__global__ __launch_bounds__(64) void k_light_paths(DevScene S, Wave Wv) {
    const BdptDev& bd = Wv.bd;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nq = Wv.n_frames * Wv.n_samples;
    if (t >= nq * bd.Ns * bd.L) return;
    const uint32_t li = t % bd.L, sub = (t / bd.L) % bd.Ns, q = t / (bd.L * bd.Ns);
    const uint32_t fr = q / Wv.n_samples, k = Wv.fsample0[fr] + (q - fr * Wv.n_samples);
    float4* out = const_cast<float4*>(bd.lv) + 3 * (size_t)t * bd.J;
    for (uint32_t j = 0; j < bd.J; ++j) out[3 * j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const DevLight& L = S.lights[li];
    const uint32_t key = path_key(Wv.seed ^ LPATH_SEED, sub * bd.L + li, k);
    Ray r = gl_light_ray(L, draw_u01(key, dim_of(0, P_LIGHT_0)), draw_u01(key, dim_of(0, P_LIGHT_1)),
                         draw_u01(key, dim_of(0, P_BSDF_0)), draw_u01(key, dim_of(0, P_BSDF_1)));
    v3 ppos = r.o, phc = mk(GL_ONE_OVER_PI, GL_ONE_OVER_PI, GL_ONE_OVER_PI);
    out[0] = make_float4(ppos.x, ppos.y, ppos.z, 1.0f);
    out[1] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    out[2] = make_float4(phc.x, phc.y, phc.z, 0.0f);
    const bool carries = L.kind == KHP_LIGHT_POINT || L.kind == KHP_LIGHT_QUAD;
    const float al = carries ? L.l : 0.0f, aq = carries ? L.q : 0.0f;
    float dist = 0.0f;
    for (uint32_t j = 1; j < bd.J; ++j) {
        if (ray_has_nan(r)) return;  // no closest hit (ray_has_nan)
        Hit h;
        PrivStack stk;
        TravStats st{0, 0, 0};
        trace_closest<false>(S, r, h, stk, st);
        if (h.slot < 0) return;  // traceLightRays: no hit ends the subpath
        ShadeCtx sc;
        khp_material mres;
        const v3 n = S.textured ? surface_at<true>(S, r, h, sc, mres) : surface_at<false>(S, r, h, sc, mres);
        const v3 pos = follow(r, h.t);
        dist = dist + length(pos - r.o);
        const float att = 1.0f / ((1.0f + dist * al) + (dist * dist) * aq);
        const v3 in = -r.d;
        v3 od = mk(0.0f, 0.0f, 0.0f), f = mk(0.0f, 0.0f, 0.0f);
        float pdf = 0.0f;
        int fl = 0;
        if (!(dot(in, n) == 0.0f)) {  // reflectance (BSDF/header.compute:48-56)
            float smp[2] = {draw_u01(key, dim_of(j, P_BSDF_0)), draw_u01(key, dim_of(j, P_BSDF_1))};
            bool valid;
            f = bsdf_sample(sc, in, n, smp, draw_u01(key, dim_of(j, P_HAIR_ALPHA)),
                            draw_u01(key, dim_of(j, P_HAIR_BETA)), od, pdf, fl, valid);
        }
        v3 hc = phc * f;
        const v3 w = pos - ppos;  // convertDensity (:280-299), previous vertex = its position
        const float ww = dot(w, w);
        if (ww == 0.0f) pdf = 0.0f;
        else pdf = pdf * fabsf(dot(n, w * sqrtf(1.0f / ww)));
        hc = hc * gclamp(fabsf(dot(od, n)) * pdf, 0.0f, 1.0f);
        if ((fl & F_EMISSIVE) == F_EMISSIVE) return;
        if (is_zero(hc) || pdf <= bd.min_pdf || att <= 0.0001f) return;
        out[3 * j] = make_float4(pos.x, pos.y, pos.z, 1.0f);
        out[3 * j + 1] = make_float4(r.d.x, r.d.y, r.d.z, 0.0f);
        out[3 * j + 2] = make_float4(hc.x, hc.y, hc.z, 0.0f);
        ppos = pos;
        phc = hc;
        r = make_ray(pos + od * bd.bounce_bias, od);
    }
}

// shadeBDPTImagePlane (pt_shade.compute:17-97; the oracle's bdpt_image_plane):
// every path connects the vertices of one subpath to its own point on the
// sensor before bounce 0.  The connections are a group of shadow records like
// k_shade's (Told = 1, no ambient: the finish adds exactly their sum) whose
// destination is the path's state at bounce 0 (queue slot = path).  Runs on
// the shadow buffers of parity 1, which bounce 0 does not use.
__global__ __launch_bounds__(256) void k_img_connect(DevScene S, Wave Wv) {
    const BdptDev& bd = Wv.bd;
    const uint32_t pid = blockIdx.x * blockDim.x + threadIdx.x;
    if (pid >= Wv.P * Wv.n_samples * Wv.n_frames) return;
    uint32_t fr, p_local, s_local;
    path_coords(Wv, pid, fr, p_local, s_local);
    const uint32_t pixel = Wv.pix[Wv.p_off + p_local];
    const uint32_t x = pixel % Wv.W, y = pixel / Wv.W;
    const uint32_t key = path_key(Wv.seed, pixel, Wv.fsample0[fr] + s_local);
    const khp_camera& cam = S.cam;
    const float u1 = draw_u01(key, dim_of(0, P_CAM_X)), u2 = draw_u01(key, dim_of(0, P_CAM_Y));
    const float s1 = ((float)x + u1) * cam.pixel_size, s2 = ((float)y + u2) * cam.pixel_size;
    const v3 sensor = (ld3(cam.bottom_left) + ld3(cam.axis_x) * s1) + ld3(cam.axis_y) * s2;
    uint32_t sp = (uint32_t)((float)bd.Ns * draw_u01(key, dim_of(IMG_BOUNCE, P_LIGHT_0)));
    uint32_t li = (uint32_t)((float)bd.L * draw_u01(key, dim_of(IMG_BOUNCE, P_LIGHT_SEL)));
    sp = sp < bd.Ns ? sp : bd.Ns - 1u;
    li = li < bd.L ? li : bd.L - 1u;
    const v3 axs = ld3(cam.axis_x) * cam.pixel_size, ays = ld3(cam.axis_y) * cam.pixel_size;
    const float a = length(cross(ays * (float)Wv.H, axs * (float)Wv.W));
    const v3 cn = normalize(cross(ays, axs));
    const uint32_t q = fr * Wv.n_samples + s_local;
    const float4* lv = bd.lv + 3 * ((((size_t)q * bd.Ns + sp) * bd.L + li) * bd.J);
    // two passes over the vertices: count the non-zero terms, then write the group
    uint32_t nv = 0;
    for (int pass = 0; pass < 2; ++pass) {
        uint32_t o = 0;
        if (pass == 1) {
            if (nv == 0) return;
            o = wave_alloc_n(nv, &Wv.shq->nsh);
        }
        bool head = true;
        for (uint32_t j = 0; j < bd.J; ++j) {
            const float4 pv = lv[3 * j];
            if (pv.w == 0.0f) continue;
            const float4 din = lv[3 * j + 1], hc = lv[3 * j + 2];
            const v3 dj = mk(din.x, din.y, din.z);
            v3 lp;
            if (bd.img == 1u) {
                // as written (pt_shade.compute:38-44): the record's ray origin + bias * its
                // direction.  Record j's ray: j = 0 (light point, 0), j = 1 (light point,
                // d0), j >= 2 (pos_{j-1} + bounce_bias * out_{j-1}, out_{j-1})
                // (lbb_construction.compute:229-235, 391-395); din_j = that direction.
                const float4 pp = lv[3 * (j >= 1u ? j - 1u : 0u)];
                const v3 org = j >= 2u ? mk(pp.x, pp.y, pp.z) + dj * bd.bounce_bias : mk(pp.x, pp.y, pp.z);
                lp = org + dj * bd.bias;
            } else {  // 2: the vertex itself, pulled back like the hit connections' target
                lp = mk(pv.x, pv.y, pv.z) - dj * bd.bounce_bias;
            }
            const v3 d = lp - sensor;
            const float t = length(d);
            const v3 dir = normalize(d);
            const float ct = dot(cn, dir);
            float we = 1.0f / ((((a * ct) * ct) * ct) * ct);
            const float npdf = (t * t) / fabsf(dot(cn, dir));
            if (ct <= 0.0f) we = 0.0f;
            const v3 cj = ((mk(hc.x, hc.y, hc.z) * we) / npdf) / (float)(j + 1);
            if (cj.x == 0.0f && cj.y == 0.0f && cj.z == 0.0f) continue;  // cannot change the sum
            if (pass == 0) {
                ++nv;
                continue;
            }
            float4* rec = Wv.sh + Wv.shs * (size_t)o++;
            rec[0] = make_float4(sensor.x, sensor.y, sensor.z, t);
            rec[1] = make_float4(dir.x, dir.y, dir.z, f_from_bits(pid));
            rec[2] = make_float4(cj.x, cj.y, cj.z, 0.0f);
            rec[3] = make_float4(1.0f, 1.0f, 1.0f, head ? (float)nv : 0.0f);
            if (head) rec[4] = make_float4(0.0f, 0.0f, 0.0f, f_from_bits(pid));  // destination: queue slot pid, parity 0
            head = false;
        }
    }
}

// One connection of a camera hit to vertex j of its chosen subpath
// (pt_shade.compute:150-199; the oracle's bdpt_connect): the connection ray
// and the contribution it adds when unoccluded.  Returns false for an invalid vertex.
__device__ __forceinline__ bool bd_connection(const DevScene& S, const BdptDev& bd, const float4* v, uint32_t j,
                                              const DevLight& L, const ShadeCtx& s, v3 loc, v3 rd, uint32_t b,
                                              Ray& sh, float& tmax, v3& cj) {
    const float4 a = v[3 * j];
    if (a.w == 0.0f) return false;
    const float4 din = v[3 * j + 1], hc = v[3 * j + 2];
    const v3 lp = mk(a.x, a.y, a.z) - mk(din.x, din.y, din.z) * bd.bounce_bias;
    v3 lc = j == 0 ? ld3(L.color) * gl_ang_att(L, lp - loc) : ld3(L.color);
    sh.o = loc + s.n * bd.bias;
    sh.d = normalize(lp - loc);
    tmax = length(lp - sh.o);
    lc = lc * fabsf(dot(sh.d, s.n));
    lc = lc * bsdf_eval(s, -rd, sh.d);
    cj = (mk(hc.x, hc.y, hc.z) * lc) / (float)(j + 1 + b);
    return true;
}

// ---- hit sorting (khp_ctx_params.shade_order = 1) ----------------------------------------
// The extension hits are grouped by shading class before k_shade, so a shade
// wave runs one BSDF's code instead of the union of several: class 0 = no
// surface hit (environment, or a light), class 1 + k = a surface whose
// material has BSDF kind k.  A counting sort over the queue: k_hit_class
// counts the classes, k_hit_scatter writes each entry's queue slot into the
// range of its class (perm).  Paths are independent and each path's state is
// updated by its own lane, so the order changes no result; the next bounce's
// queues come out grouped the same way.
// ---- ray sorting (khp_ctx_params.sort_from): a bounce's queue regrouped by origin cell ----
// Deep bounces start inside the hairball in every direction, and a wave's 64
// rays (neighbouring queue slots) come from paths that diverged bounces ago, so
// they fetch unrelated subtrees.  A counting sort by the Morton cell of the ray
// origin (32^3 cells over the root box) lays the queue out so that a claim block
// holds rays that start close together, and whose near subtrees therefore share
// L2 lines.  Which lane traces which ray changes no result (every entry is
// claimed exactly once and written to its own slot).  All counts stay on the
// device: k_rsort_count (cells), k_rsort_scan (cell offsets), k_rsort_scatter
// (the regrouped ray columns and the state indirection).
constexpr uint32_t RS_LOG = 5;   // cells per axis = 2^RS_LOG (16^3 cells measured the same)
constexpr uint32_t RS_CELLS = 1u << (3 * RS_LOG);
// k_rsort_count / k_rsort_scatter privatise the cell histogram in LDS: 2^15 cells
// are 128 KiB, which only gfx950's 160 KiB per workgroup holds (64 KiB before it)
static_assert(RS_CELLS * sizeof(uint32_t) <= 160 * 1024, "ray-sort histogram exceeds gfx950's LDS per workgroup");
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "render.hip is written for gfx950 (MI355X): k_rsort_* need 128 KiB of LDS per workgroup (RS_LOG 4 fits 16 KiB)"
#endif
__device__ __forceinline__ uint32_t rs_spread(uint32_t v) {   // 5 bits -> every third bit
    v &= 31u;
    v = (v | (v << 8)) & 0x100Fu;
    v = (v | (v << 4)) & 0x10C3u;
    v = (v | (v << 2)) & 0x1249u;
    return v;
}
__device__ __forceinline__ uint32_t rs_cell(const DevScene& S, float ox, float oy, float oz) {
    const float* b = S.root_box;
    auto q = [](float o, float lo, float hi) {
        constexpr float R = (float)(1u << RS_LOG);
        const float f = (o - lo) / (hi - lo) * R;   // NaN -> 0 below
        return (uint32_t)(f >= R - 1.0f ? R - 1.0f : (f > 0.0f ? f : 0.0f));
    };
    return rs_spread(q(ox, b[0], b[3])) | (rs_spread(q(oy, b[1], b[4])) << 1) | (rs_spread(q(oz, b[2], b[5])) << 2);
}
// Cell counts are privatised per block in LDS (one 1024-thread block per CU,
// the 2^15 counters in 128 KiB): a block adds its slice of the queue there and
// then touches the global counter of each cell it saw once.  Same-address
// global atomics per ray serialise in L2 and cost ~1 ns per ray (measured).
constexpr uint32_t RS_THREADS = 1024;
constexpr uint64_t RS_AUTO_BYTES = 64ull << 20;   // automatic regrouping from this tree size (node records)
__device__ __forceinline__ void rs_slice(uint32_t n, uint32_t& a, uint32_t& b) {
    const uint32_t per = (n + gridDim.x - 1) / gridDim.x;
    a = blockIdx.x * per;
    b = a + per < n ? a + per : n;
    a = a < n ? a : n;
}
// count: the cell of every queued ray (keys[v], by virtual index) and the cell totals
__global__ __launch_bounds__(RS_THREADS) void k_rsort_count(DevScene S, Wave Wv, int q, uint32_t* hist,
                                                            uint32_t* keys) {
    __shared__ uint32_t lh[RS_CELLS];
    const uint32_t nf = Wv.cnt->nq[q], n = nf + Wv.cnt->nqb[q];
    for (uint32_t c = threadIdx.x; c < RS_CELLS; c += RS_THREADS) lh[c] = 0u;
    __syncthreads();
    uint32_t a, b;
    rs_slice(n, a, b);
    for (uint32_t v = a + threadIdx.x; v < b; v += RS_THREADS) {
        const uint32_t i = q_phys(v, nf, Wv.cap);
        const uint32_t c = rs_cell(S, Wv.qo[q][0][i], Wv.qo[q][1][i], Wv.qo[q][2][i]);
        keys[v] = c;
        atomicAdd(&lh[c], 1u);
    }
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < RS_CELLS; c += RS_THREADS)
        if (lh[c]) atomicAdd(&hist[c], lh[c]);
}
// exclusive prefix of the cell counts (one block): cursor[c] = first output position of cell c
__global__ __launch_bounds__(1024) void k_rsort_scan(const uint32_t* hist, uint32_t* cursor) {
    __shared__ uint32_t part[1024];
    constexpr uint32_t PER = RS_CELLS / 1024;
    const uint32_t t = threadIdx.x;
    uint32_t sum = 0;
    for (uint32_t k = 0; k < PER; ++k) sum += hist[t * PER + k];
    part[t] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {   // inclusive Hillis-Steele scan
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - sum;
    for (uint32_t k = 0; k < PER; ++k) {
        cursor[t * PER + k] = run;
        run += hist[t * PER + k];
    }
}
// scatter: each block reserves one range per cell it holds, then writes its rays'
// columns and their state slots there (reads coalesced; the writes come in runs,
// one per cell and block).  Regrouped entry j goes to the physical slot virtual
// index j had, so the queue's front / back counts still describe it; its state
// stays at slot qsrc[j].  (A permutation plus a gather pass with scattered reads
// measured 0.06 ms per frame slower, profiles/r05ab_sort_scatter_ab.txt.)
__global__ __launch_bounds__(RS_THREADS) void k_rsort_scatter(Wave Wv, int q, const uint32_t* keys, uint32_t* cursor,
                                                              float* cols, uint32_t* qsrc) {
    __shared__ uint32_t lh[RS_CELLS];
    const uint32_t nf = Wv.cnt->nq[q], n = nf + Wv.cnt->nqb[q];
    const size_t cap = Wv.cap;
    for (uint32_t c = threadIdx.x; c < RS_CELLS; c += RS_THREADS) lh[c] = 0u;
    __syncthreads();
    uint32_t a, b;
    rs_slice(n, a, b);
    for (uint32_t v = a + threadIdx.x; v < b; v += RS_THREADS) atomicAdd(&lh[keys[v]], 1u);
    __syncthreads();
    for (uint32_t c = threadIdx.x; c < RS_CELLS; c += RS_THREADS)
        if (lh[c]) lh[c] = atomicAdd(&cursor[c], lh[c]);
    __syncthreads();
    for (uint32_t v = a + threadIdx.x; v < b; v += RS_THREADS) {
        const uint32_t src = q_phys(v, nf, Wv.cap);
        const uint32_t dst = q_phys(atomicAdd(&lh[keys[v]], 1u), nf, Wv.cap);
        for (int k = 0; k < 3; ++k) {
            cols[k * cap + dst] = Wv.qo[q][k][src];
            cols[(3 + k) * cap + dst] = Wv.qd[q][k][src];
        }
        reinterpret_cast<uint32_t*>(cols)[6 * cap + dst] = Wv.qpid[q][src];
        qsrc[dst] = src;
    }
}
constexpr uint32_t NCLS = 1 + KHP_BSDF_COUNT;
static_assert(NCLS <= 16, "hit classes");
__device__ __forceinline__ uint32_t hit_class(const DevScene& S, int32_t slot) {
    return slot < 0 ? 0u : 1u + (uint32_t)S.mats[S.aux[slot].mat].bsdf;
}
__global__ __launch_bounds__(256) void k_hit_class(DevScene S, Wave Wv, int cur) {
    __shared__ uint32_t h[16];
    const uint32_t nf = Wv.cnt->nq[cur], n = nf + Wv.cnt->nqb[cur];
    if (threadIdx.x < 16) h[threadIdx.x] = 0;
    __syncthreads();
    for (uint32_t iv = blockIdx.x * blockDim.x + threadIdx.x; iv < n; iv += gridDim.x * blockDim.x) {
        const uint32_t k = hit_class(S, Wv.hslot[q_phys(iv, nf, Wv.cap)]);
        Wv.hkey[iv] = (uint8_t)k;
        atomicAdd(&h[k], 1u);
    }
    __syncthreads();
    if (threadIdx.x < NCLS && h[threadIdx.x]) atomicAdd(&Wv.hcls[threadIdx.x], h[threadIdx.x]);
}
__global__ __launch_bounds__(256) void k_hit_scatter(Wave Wv, int cur) {
    __shared__ uint32_t base[16], cnt[16], off[16];
    const uint32_t nf = Wv.cnt->nq[cur], n = nf + Wv.cnt->nqb[cur];
    if (threadIdx.x < 16) {
        uint32_t b = 0;
        for (uint32_t k = 0; k < threadIdx.x && k < NCLS; ++k) b += Wv.hcls[k];
        base[threadIdx.x] = b;
    }
    for (uint32_t t0 = blockIdx.x * blockDim.x; t0 < n; t0 += gridDim.x * blockDim.x) {
        const uint32_t iv = t0 + threadIdx.x;
        if (threadIdx.x < 16) cnt[threadIdx.x] = 0;
        __syncthreads();
        const uint32_t k = iv < n ? Wv.hkey[iv] : 0u;
        const uint32_t local = iv < n ? atomicAdd(&cnt[k], 1u) : 0u;
        __syncthreads();
        if (threadIdx.x < NCLS && cnt[threadIdx.x]) off[threadIdx.x] = atomicAdd(&Wv.hcls[16 + threadIdx.x], cnt[threadIdx.x]);
        __syncthreads();
        if (iv < n) Wv.perm[base[k] + off[k] + local] = q_phys(iv, nf, Wv.cap);
        __syncthreads();
    }
}

// Hit texcoord (Cylinder::calcTcoord, Cylinder.cpp:239-260; Triangle::calcTcoord,
// Triangle.cpp:250-254) and the material with its textured parameters resolved.
// m holds the material's values on entry (resolve_material overwrites the textured ones).
__device__ __forceinline__ void textured_material(const DevScene& S, const Aux& ax, const float4* pr, v3 loc,
                                               const ShadeCtx& s, float bu, float bv, khp_material& out) {
    float tu, tv;
    if (ax.flags & 1u) {
        const float4 c0 = pr[0];
        const v3 Q = loc - mk(c0.x, c0.y, c0.z);
        const float qu = dot(Q, s.U), qv = dot(Q, s.V), qw = dot(Q, s.W);
        const float rr = c0.w - pr[1].w * qv;
        const float tmp = gclamp(qw / rr, -1.0f, 1.0f);
        const float phi = qu < 0.0f ? 2.0f * PIF - k_acosf(tmp) : k_acosf(tmp);
        tu = phi / 2.0f / PIF;
        tv = qv / S.cone_h[ax.obj - S.n_tris];
    } else {
        const float* tc = S.tri_uv + 6 * (size_t)ax.obj;
        const float bx = (1.0f - bu) - bv;
        tu = (bx * tc[0] + bu * tc[2]) + bv * tc[4];
        tv = (bx * tc[1] + bu * tc[3]) + bv * tc[5];
    }
    resolve_material(S, ax.mat, tu, tv, out);
}

// ---- shade: traceRay light test + shaders (CPU_PathTracer.cpp:141-208; SimpleShader.h;
//      MarschnerHairShader.h; LightShader.h; EnvironmentShader.h) ------------------------
// Block-aggregated queue allocation for the two outputs of k_shade: one
// atomic per 256-thread block and queue instead of one per wave.  Device-scope
// atomics on a single counter serialize across the XCDs; with wave-level
// allocation k_shade spent most of its time waiting on them.
struct BlockAlloc2 {
    uint32_t wcnt[2][4];
    uint32_t base[2];
};
__device__ __forceinline__ void block_alloc2(bool p0, bool p1, uint32_t* c0, uint32_t* c1, BlockAlloc2& sh,
                                             uint32_t& i0, uint32_t& i1) {
    const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
    const unsigned long long m0 = __ballot(p0), m1 = __ballot(p1);
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (lane == 0) {
        sh.wcnt[0][wid] = (uint32_t)__popcll(m0);
        sh.wcnt[1][wid] = (uint32_t)__popcll(m1);
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const uint32_t q = threadIdx.x;
        const uint32_t tot = sh.wcnt[q][0] + sh.wcnt[q][1] + sh.wcnt[q][2] + sh.wcnt[q][3];
        sh.base[q] = tot ? atomicAdd(q == 0 ? c0 : c1, tot) : 0u;
    }
    __syncthreads();
    uint32_t o0 = sh.base[0], o1 = sh.base[1];
    for (uint32_t w = 0; w < wid; ++w) {
        o0 += sh.wcnt[0][w];
        o1 += sh.wcnt[1][w];
    }
    i0 = o0 + (uint32_t)__popcll(m0 & lt);
    i1 = o1 + (uint32_t)__popcll(m1 & lt);
    __syncthreads();  // sh is reused by the next iteration
}

// k_shade's block: 512 threads (8 waves).  Its queue allocation is one device atomic
// per output kind per block iteration; 512-thread blocks halve those against 256 and
// measured +1.4% (default bench) / +1.6% (driver's command) on the whole frame; 128
// threads doubled them and lost 4% (profiles/r04ah_shade_block.json).  Round 6:
// 1024 threads for the untextured instances without the light-path variant (101 /
// 105 VGPRs, no scratch) -- a block's surviving rays then fill one run of the next
// queue from 16 pixels' paths, and bounce 1's k_extend takes 6.85 instead of 7.06
// ms per frame (+0.3% on the driver's command, profiles/r06zx_shade_block_1024_ab.txt);
// the textured and light-path instances would spill at 1024 and keep 512.
#ifndef KHP_SHADE_BLOCK
#define KHP_SHADE_BLOCK 512
#endif
#ifndef KHP_SHADE_BLOCK_PLAIN
#define KHP_SHADE_BLOCK_PLAIN 1024
#endif
template <bool TEX, bool BD>
constexpr uint32_t shade_block() { return (!TEX && !BD) ? KHP_SHADE_BLOCK_PLAIN : KHP_SHADE_BLOCK; }
// Four outputs (next-bounce rays and shadow rays, each front or back): a lane
// sets at most one of p0/p1 and one of p2/p3; i01 / i23 is its index in the
// queue it was counted in.
template <uint32_t NW>   // waves per block
struct BlockAlloc4 {
    uint32_t wcnt[4][NW];
    uint32_t base[4];
};
template <uint32_t NW>
__device__ __forceinline__ void block_alloc4(bool p0, bool p1, bool p2, bool p3, uint32_t* c0, uint32_t* c1,
                                             uint32_t* c2, uint32_t* c3, BlockAlloc4<NW>& sh, uint32_t& i01,
                                             uint32_t& i23) {
    const uint32_t lane = lane_id(), wid = threadIdx.x >> 6;
    const unsigned long long m[4] = {__ballot(p0), __ballot(p1), __ballot(p2), __ballot(p3)};
    const unsigned long long lt = (1ull << lane) - 1ull;
    if (lane == 0)
        for (int q = 0; q < 4; ++q) sh.wcnt[q][wid] = (uint32_t)__popcll(m[q]);
    __syncthreads();
    if (threadIdx.x < 4) {
        const uint32_t q = threadIdx.x;
        uint32_t tot = 0;
        for (uint32_t w = 0; w < NW; ++w) tot += sh.wcnt[q][w];
        uint32_t* ctr = q == 0 ? c0 : q == 1 ? c1 : q == 2 ? c2 : c3;
        sh.base[q] = tot ? atomicAdd(ctr, tot) : 0u;
    }
    __syncthreads();
    uint32_t o[4] = {sh.base[0], sh.base[1], sh.base[2], sh.base[3]};
    for (uint32_t w = 0; w < wid; ++w)
        for (int q = 0; q < 4; ++q) o[q] += sh.wcnt[q][w];
    i01 = p0 ? o[0] + (uint32_t)__popcll(m[0] & lt) : o[1] + (uint32_t)__popcll(m[1] & lt);
    i23 = p2 ? o[2] + (uint32_t)__popcll(m[2] & lt) : o[3] + (uint32_t)__popcll(m[3] & lt);
    __syncthreads();  // sh is reused by the next iteration
}

// TEX: the scene has textured materials or an environment map (a separate
// instantiation, so untextured scenes keep k_shade's registers).
#ifndef KHP_SHADE_WAVES
#define KHP_SHADE_WAVES 1   // min waves per SIMD for k_shade's register budget (1: unconstrained)
#endif
template <bool TEX, bool BD, uint32_t KINDS = 0xFFFFFFFFu>
__global__ __launch_bounds__((shade_block<TEX, BD>()), KHP_SHADE_WAVES) void k_shade(DevScene S, Wave Wv, int cur, uint32_t bounce) {
    const uint32_t nf = Wv.cnt->nq[cur], n = nf + Wv.cnt->nqb[cur];
    const int nxt = cur ^ 1;
    const bool last = bounce + 1 >= Wv.depth;
    const uint32_t stride = gridDim.x * blockDim.x;
    __shared__ BlockAlloc4<shade_block<TEX, BD>() / 64> balloc;
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += stride) {
        const uint32_t iv = base + threadIdx.x;
        bool active = iv < n;
        const uint32_t i = !active ? 0u : Wv.perm ? Wv.perm[iv] : q_phys(iv, nf, Wv.cap);
        const bool heavy = active && Wv.heavy[i] != 0;
        bool emit_ray = false, emit_sh = false;
        Ray nr;
        nr.o = nr.d = mk(0, 0, 0);
        uint32_t pid = 0;
        // shadow record payload
        Ray shr;
        shr.o = shr.d = mk(0, 0, 0);
        float sh_tmax = 0.0f;
        v3 lc = mk(0, 0, 0), Told = mk(0, 0, 0), AT = mk(0, 0, 0), ET = mk(0, 0, 0);
        bool has_emit = false;
        uint32_t bd_head = 0xFFFFFFFFu;  // BD: the group's head record (its rec[4] is written with the destination)
        float4 tfo = make_float4(0.0f, 0.0f, 0.0f, 0.0f), cko = tfo;  // the path state after this bounce
        if (active) {
            Ray r;
            float4 tf, ck;
            if (bounce == 0 && Wv.cam0) {  // the bounce-0 state k_generate would have queued
                uint32_t key0;
                pid = i;
                r = camera_path(S, Wv, i, key0);
                tf = make_float4(1.0f, 1.0f, 1.0f, f_from_bits(0u));
                ck = make_float4(0.0f, 0.0f, 0.0f, f_from_bits(key0));
            } else {
                pid = Wv.qpid[cur][i];
                r.o = mk(Wv.qo[cur][0][i], Wv.qo[cur][1][i], Wv.qo[cur][2][i]);
                r.d = mk(Wv.qd[cur][0][i], Wv.qd[cur][1][i], Wv.qd[cur][2][i]);
                const uint32_t si = Wv.qsrc ? Wv.qsrc[i] : i;
                tf = Wv.TFq[cur][si];
                ck = Wv.CKq[cur][si];
            }
            float lambda = Wv.ht[i];
            int32_t slot = Wv.hslot[i];
            v3 T = mk(tf.x, tf.y, tf.z);
            v3 C = mk(ck.x, ck.y, ck.z);
            int flags = (int)bits_from_f(tf.w);
            uint32_t key = bits_from_f(ck.w);
            // KIRK's linear ray-light test (CPU_PathTracer.cpp:185-208)
            float t_lights = FLT_MAX_;
            int t_index = -1;
            for (int li = 0; li < S.n_lights; ++li) {
                float t = FLT_MAX_;
                if (light_isect(S.lights[li], r, t)) {
                    t_lights = gmin(t_lights, t);
                    t_index = (t == t_lights) ? li : t_index;
                }
            }
            bool light_hit = false;
            if (t_lights < lambda) {
                lambda = t_lights;
                light_hit = true;
            }
            if (lambda == FLT_MAX_) {  // EnvironmentShader::shade
                C = C + (TEX ? env_color(S, r.d) : mk(S.env.color[0], S.env.color[1], S.env.color[2])) * T;
                T = mk(0, 0, 0);
            } else if (light_hit) {    // LightShader::shade
                C = C + light_emit(S.lights[t_index], r.d) * T;
                T = mk(0, 0, 0);
            } else {
                // normal and hair frame (Cylinder::calcNormal / Triangle::calcNormal), material
                ShadeCtx s;
                khp_material mres;
                const Hit hh{lambda, slot, 0.0f, 0.0f};  // u, v: surface_at recomputes them
                const v3 nrm = surface_at<TEX>(S, r, hh, s, mres);
                const v3 loc = follow(r, lambda);
                const khp_material* m = s.m;
                float h0 = draw_u01(key, dim_of(bounce, P_HAIR_ALPHA)), h1 = draw_u01(key, dim_of(bounce, P_HAIR_BETA));
                v3 counter = -normalize(r.d);
                // NEE setup: SimpleShader::calcDirectLight (SimpleShader.h:101-152) and
                // MarschnerHairShader::calcDirectLight (MarschnerHairShader.h:87-138)
                bool need_shadow = false;
                if (!BD && S.n_lights > 0) {
                    int li = (int)((double)draw_u01(key, dim_of(bounce, P_LIGHT_SEL)) * (double)S.n_lights);
                    const DevLight& L = S.lights[li];
                    float att;
                    Ray h2l = light_dir(L, loc, draw_u01(key, dim_of(bounce, P_LIGHT_0)),
                                        draw_u01(key, dim_of(bounce, P_LIGHT_1)), att);
                    v3 lightpos = h2l.o + h2l.d;
                    h2l.o = h2l.o + faceforward(nrm, h2l.o - lightpos, nrm) * 1e-4f;
                    h2l.d = normalize(h2l.d);
                    if (L.color[0] > 0.0f || L.color[1] > 0.0f || L.color[2] > 0.0f) {
                        v3 f = bsdf_eval(s, h2l.d, -r.d);
                        float ad = fabsf(dot(h2l.d, nrm));
                        lc = mk(L.color[0] * ((att * f.x) * ad), L.color[1] * ((att * f.y) * ad),
                                L.color[2] * ((att * f.z) * ad));
                        sh_tmax = length(lightpos - h2l.o);
                        shr = h2l;
                        need_shadow = true;
                    }
                }
                v3 ev = bsdf_eval(s, nrm, nrm);
                v3 amb = mk(S.env.ambient[0], S.env.ambient[1], S.env.ambient[2]) * (ev * ONE_OVER_PI);
                Told = T;
                AT = amb * T;
                bool add_now = true;  // colour add not deferred to the shadow kernel
                if (m->shader == KHP_SHADER_MARSCHNER_HAIR) {  // MarschnerHairShader::shade
                    float smp[2] = {0.0f, 0.0f};
                    v3 out;
                    float pdf = 0.0f;
                    bool valid;
                    v3 refl = bsdf_sample<KINDS>(s, counter, nrm, smp, h0, h1, out, pdf, flags, valid);
                    v3 off = out * 1e-4f;
                    if (!(flags & F_SPECULAR)) off = faceforward(-(nrm * 1e-4f), nrm, out);
                    nr = make_ray(loc + off, out);
                    if ((flags & F_CYL_T) || (flags & F_CYL_TR)) {
                        need_shadow = false;
                        add_now = false;
                    } else {
                        if (is_zero(refl) || pdf <= 1E-4f || gmax(T.x, gmax(T.y, T.z)) < 0.01f) T = mk(0, 0, 0);
                        else T = T * ((refl * 3.0f) * fabsf(k_cosf(smp[0])));
                    }
                } else {  // SimpleShader::shade
                    float smp[2] = {draw_u01(key, dim_of(bounce, P_BSDF_0)), draw_u01(key, dim_of(bounce, P_BSDF_1))};
                    v3 out;
                    float pdf = 0.0f;
                    int fl = 0;
                    bool valid;
                    v3 refl = bsdf_sample<KINDS>(s, counter, nrm, smp, h0, h1, out, pdf, fl, valid);
                    if (is_zero(refl) || pdf <= 1E-4f || gmax(T.x, gmax(T.y, T.z)) < 0.01f) {
                        T = mk(0, 0, 0);
                    } else if ((fl & F_EMISSIVE) == F_EMISSIVE) {
                        has_emit = true;
                        ET = mk(m->emission[0], m->emission[1], m->emission[2]) * T;
                        T = mk(0, 0, 0);
                    } else {
                        float ad = fabsf(dot(out, nrm));
                        T = T * ((refl * ad) / pdf);
                        flags = fl;
                        v3 off = out * 1e-4f;
                        if ((fl & F_SPECULAR) != F_SPECULAR) off = faceforward(-(nrm * 1e-4f), nrm, out);
                        nr = make_ray(loc + off, out);
                    }
                }
                if (add_now && BD) {
                    // pt_shade.compute:146-201: connect to every valid vertex of one subpath.
                    // Contributions that are +-0 in every channel cannot change the sum
                    // (it starts at +0), so they get no connection ray.
                    uint32_t nv = 0, sp = 0, li = 0;
                    const float4* lv = nullptr;
                    if (S.n_lights > 0) {
                        const BdptDev& bd = Wv.bd;
                        sp = (uint32_t)((float)bd.Ns * draw_u01(key, dim_of(bounce, P_LIGHT_0)));
                        li = (uint32_t)((float)bd.L * draw_u01(key, dim_of(bounce, P_LIGHT_SEL)));
                        sp = sp < bd.Ns ? sp : bd.Ns - 1u;
                        li = li < bd.L ? li : bd.L - 1u;
                        uint32_t fr, p_local, s_local;
                        path_coords(Wv, pid, fr, p_local, s_local);
                        const uint32_t q = fr * Wv.n_samples + s_local;
                        lv = bd.lv + 3 * ((((size_t)q * bd.Ns + sp) * bd.L + li) * bd.J);
                        for (uint32_t j = 0; j < bd.J; ++j) {
                            Ray sh;
                            float tm;
                            v3 cj;
                            if (bd_connection(S, bd, lv, j, S.lights[li], s, loc, r.d, bounce, sh, tm, cj) &&
                                !(cj.x == 0.0f && cj.y == 0.0f && cj.z == 0.0f))
                                ++nv;
                        }
                    }
                    if (nv == 0) {
                        v3 acc = (mk(0, 0, 0) + mk(0, 0, 0) * Told) + AT;
                        if (has_emit) acc = acc + ET;
                        C = C + acc;
                    } else {  // the colour add is left to the group's finish
                        const BdptDev& bd = Wv.bd;
                        uint32_t o = wave_alloc_n(nv, &Wv.shq->nsh);
                        bool head = true;
                        for (uint32_t j = 0; j < bd.J; ++j) {
                            Ray sh;
                            float tm;
                            v3 cj;
                            if (!bd_connection(S, bd, lv, j, S.lights[li], s, loc, r.d, bounce, sh, tm, cj) ||
                                (cj.x == 0.0f && cj.y == 0.0f && cj.z == 0.0f))
                                continue;
                            float4* rec = Wv.sh + Wv.shs * (size_t)o++;
                            rec[0] = make_float4(sh.o.x, sh.o.y, sh.o.z, tm);
                            rec[1] = make_float4(sh.d.x, sh.d.y, sh.d.z, f_from_bits(pid));
                            rec[2] = make_float4(cj.x, cj.y, cj.z, has_emit ? 1.0f : 0.0f);
                            rec[3] = make_float4(Told.x, Told.y, Told.z, head ? (float)nv : 0.0f);
                            if (head) {
                                bd_head = o - 1u;
                                if (has_emit) rec[5] = make_float4(ET.x, ET.y, ET.z, 0.0f);
                            }
                            head = false;
                        }
                    }
                } else if (add_now) {
                    if (need_shadow && !(lc.x == 0.0f && lc.y == 0.0f && lc.z == 0.0f)) {
                        emit_sh = true;  // colour is added by k_shadow
                    } else if (need_shadow) {
                        // Zero light colour (31.7% of the metric row's shadow rays,
                        // measured with a debug counter): shadow_finish_one's lc * (occ ? 0 : 1)
                        // is lc itself for +-0, so the any-hit result cannot change the
                        // colour and the ray is not traced.  Same operations as the finish.
                        v3 dl = mk(0, 0, 0) + lc * 1.0f;
                        v3 acc = (mk(0, 0, 0) + dl * Told) + AT;
                        if (has_emit) acc = acc + ET;
                        C = C + acc;
                    } else {
                        v3 acc = (mk(0, 0, 0) + mk(0, 0, 0) * Told) + AT;
                        if (has_emit) acc = acc + ET;
                        C = C + acc;
                    }
                }
            }
            // (with a deferred add -- emit_sh or a BD group -- C is unchanged here and the
            // shadow finish adds this bounce's term to wherever the state goes)
            tfo = make_float4(T.x, T.y, T.z, f_from_bits((uint32_t)flags));
            cko = make_float4(C.x, C.y, C.z, ck.w);
            emit_ray = !last && !is_zero(T) && !is_zero(nr.d);
        }
        uint32_t qi, si;
        block_alloc4(emit_ray && heavy, emit_ray && !heavy, emit_sh && heavy, emit_sh && !heavy,
                     &Wv.cnt->nq[nxt], &Wv.cnt->nqb[nxt], &Wv.shq->nsh, &Wv.shq->nshb, balloc, qi, si);
        qi = heavy ? qi : Wv.cap - 1u - qi;
        si = heavy ? si : Wv.cap - 1u - si;
        // The path state moves with the ray: to the next queue slot (coalesced
        // with the ray's own columns), or, when the path ends, to its final
        // colour CK[pid].  A deferred colour add is told where the state went.
        const uint32_t dest = emit_ray ? qi : (0x80000000u | pid);
        if (emit_ray) {
            Wv.qo[nxt][0][qi] = nr.o.x; Wv.qo[nxt][1][qi] = nr.o.y; Wv.qo[nxt][2][qi] = nr.o.z;
            Wv.qd[nxt][0][qi] = nr.d.x; Wv.qd[nxt][1][qi] = nr.d.y; Wv.qd[nxt][2][qi] = nr.d.z;
            Wv.qpid[nxt][qi] = pid;
            Wv.TFq[nxt][qi] = tfo;
            Wv.CKq[nxt][qi] = cko;
        } else if (active) {
            Wv.CK[pid] = cko;
        }
        if (emit_sh) {
            // The finish adds one of two values: the light's term if the shadow ray is
            // unoccluded, none if it is -- both computed here with the finish's own
            // operations (lc * (occ ? 0 : 1), then (0 + dl * Told) + AT [+ ET]), so the
            // record is 64 B instead of 96 and the finish reads one of them
            float4* rec = Wv.sh + Wv.shs * (size_t)si;
            rec[0] = make_float4(shr.o.x, shr.o.y, shr.o.z, sh_tmax);
            rec[1] = make_float4(shr.d.x, shr.d.y, shr.d.z, f_from_bits(dest));
            const v3 dl_u = mk(0, 0, 0) + lc * 1.0f, dl_o = mk(0, 0, 0) + lc * 0.0f;
            v3 add_u = (mk(0, 0, 0) + dl_u * Told) + AT, add_o = (mk(0, 0, 0) + dl_o * Told) + AT;
            if (has_emit) {
                add_u = add_u + ET;
                add_o = add_o + ET;
            }
            rec[2] = make_float4(add_u.x, add_u.y, add_u.z, 0.0f);
            rec[3] = make_float4(add_o.x, add_o.y, add_o.z, 0.0f);
        }
        if (BD && bd_head != 0xFFFFFFFFu) Wv.sh[Wv.shs * (size_t)bd_head + 4] = make_float4(AT.x, AT.y, AT.z, f_from_bits(dest));
    }
}

// ---- shadow: BVH::isIntersection (k_shadow), then the light occlusion loop and
//      the deferred colour add (k_shadow_finish, SimpleShader.h:131-148) ---------------
// k_shadow_finish: one shadow record per lane, streaming; kept out of the
// traversal kernel so k_shadow's registers go to traversal only.
// The light occlusion loop and colour add of one shadow record (SimpleShader.h:131-148).
// Where shade left a path's state: the next queue slot (parity nxt), or, high bit set, the final colour of path i.
__device__ __forceinline__ float4* state_dest(const Wave& Wv, int nxt, uint32_t dest) {
    return (dest & 0x80000000u) ? Wv.CK + (dest & 0x7FFFFFFFu) : Wv.CKq[nxt] + dest;
}

__device__ __forceinline__ void shadow_finish_one(const DevScene& S, const Wave& Wv, int nxt, uint32_t i, bool occ) {
    const float4* rec = Wv.sh + Wv.shs * (size_t)i;
    const float4 b = rec[1];
    if (!occ) {   // KIRK's light occlusion loop (the any-hit result came from k_shadow)
        const float4 a = rec[0];
        Ray r;
        r.o = mk(a.x, a.y, a.z);
        r.d = mk(b.x, b.y, b.z);
        const float tmax = a.w;
        for (int li = 0; li < S.n_lights; ++li) {
            float t;
            if (light_isect(S.lights[li], r, t) && (t < tmax)) {
                occ = true;
                break;
            }
        }
    }
    const float4 acc = rec[occ ? 3 : 2];   // k_shade's precomputed add for this outcome
    float4* dst = state_dest(Wv, nxt, bits_from_f(b.w));
    const float4 ck = *dst;
    *dst = make_float4(ck.x + acc.x, ck.y + acc.y, ck.z + acc.z, ck.w);
}

// BD: the records of a light-path connection group (one path, one bounce) are
// consecutive in the front part; the head (rec[3].w = group size) adds the
// unoccluded contributions in vertex order (the oracle's bdpt_connect).
__device__ __forceinline__ void connection_group_finish(const DevScene& S, const Wave& Wv, int nxt, uint32_t i) {
    const float4* rec = Wv.sh + Wv.shs * (size_t)i;
    const float4 d = rec[3];
    if (d.w == 0.0f) return;  // not a group head
    const uint32_t nv = (uint32_t)d.w;
    const uint32_t pid = bits_from_f(rec[1].w);
    v3 dl = mk(0, 0, 0);
    for (uint32_t m = 0; m < nv; ++m) {
        const float4* q = rec + Wv.shs * (size_t)m;
        const float4 a = q[0], b = q[1], c = q[2];
        bool occ = Wv.vis[i + m] != 0;
        if (!occ) {
            Ray r;
            r.o = mk(a.x, a.y, a.z);
            r.d = mk(b.x, b.y, b.z);
            for (int li = 0; li < S.n_lights; ++li) {
                float t;
                if (light_isect(S.lights[li], r, t) && (t < a.w)) {
                    occ = true;
                    break;
                }
            }
        }
        if (!occ) dl = dl + mk(c.x, c.y, c.z);
    }
    const float4 e = rec[4];
    v3 acc = (mk(0, 0, 0) + dl * mk(d.x, d.y, d.z)) + mk(e.x, e.y, e.z);
    if (rec[2].w != 0.0f) {
        const float4 f = rec[5];
        acc = acc + mk(f.x, f.y, f.z);
    }
    (void)pid;
    float4* dst = state_dest(Wv, nxt, bits_from_f(e.w));
    const float4 ck = *dst;
    *dst = make_float4(ck.x + acc.x, ck.y + acc.y, ck.z + acc.z, ck.w);
}

template <bool BD>
__global__ __launch_bounds__(256) void k_shadow_finish(DevScene S, Wave Wv, int nxt) {
    const uint32_t nf = Wv.shq->nsh, n = nf + Wv.shq->nshb;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&Wv.cnt->sh_rays, (unsigned long long)n);
    for (uint32_t iv = blockIdx.x * blockDim.x + threadIdx.x; iv < n; iv += gridDim.x * blockDim.x) {
        const uint32_t i = q_phys(iv, nf, Wv.cap);
        if (BD) connection_group_finish(S, Wv, nxt, i);
        else shadow_finish_one(S, Wv, nxt, i, Wv.vis[i] != 0);
    }
}

// WIDE: the two-level records (traverse.h iterw) instead of the 64-B loop.
template <bool STATS, bool WIDE = false, bool TOP = false>
__global__ __launch_bounds__(TRAV_BLOCK, TRAV_WAVES) void k_shadow(DevScene S, Wave Wv, SpillArea spill) {
    extern __shared__ uint32_t lds[];
    const uint32_t nf = Wv.shq->nsh, nb = Wv.shq->nshb;
    TravStack<STATS, TOP> stk;
    stk.init(lds, spill.base, spill.stride);
    if (TOP) stk.stage_top(S.top);
    TravStats st{0, 0, 0};
    TravRay tr;
    Cur c{0u, 0.0f, 0.0f, false};
    LeafCur lf{0u, 0u, 0.0f, 0.0f, 0.0f, 0.0f, -1};
    unsigned long long wit = 0, wbusy = 0;  // STATS: wave iterations, busy lanes
    float tmax = 0.0f;
    uint32_t mode = 0u;
    bool has = false, exhausted = false;
    Claimer cl;
    cl.init(Wv.shq->fetch, nf, nb, Wv.cap);
    uint32_t idx = 0;
    for (;;) {
        unsigned long long idle = __ballot(!has);
        if (!exhausted && __popcll(idle) >= REFILL) {
            uint32_t my;
            const bool got = cl.claim(idle, my, exhausted);
            if (!has && got && cl.phys(my, idx)) {
                const float4* rec = Wv.sh + Wv.shs * (size_t)idx;
                float4 a = rec[0], b = rec[1];
                Ray r;
                r.o = mk(a.x, a.y, a.z);
                r.d = mk(b.x, b.y, b.z);
                tmax = a.w;
                trav_setup(tr, r);
                lf.left = 0;
                if (!STATS && x_slab_nan(tr)) {  // the whole-tree walk, answered exactly (any_hit_x_nan)
                    has = false;
                    Wv.vis[idx] = any_hit_x_nan(S, r) ? 1 : 0;
                } else {
                    has = trav2_begin<STATS>(S, tr, tmax, stk, mode, c, lf, st);
                    if (!has) Wv.vis[idx] = 0;
                }
            }
        }
        unsigned long long act = __ballot(has);
        if (act == 0) {
            if (exhausted) break;
            continue;
        }
        for (;;) {
            if (STATS) {
                unsigned long long wm = __ballot(has && (mode == M_NODE || mode == M_LEAF));
                ++wit;
                wbusy += (uint32_t)__popcll(wm);
            }
            if (has) {
                bool occ = false;
                Hit hu_{0.0f, -1, 0.0f, 0.0f};
                const bool fin = WIDE ? iterw<true, STATS>(S, tr, hu_, tmax, stk, mode, c, lf, st, occ)
                                      : iter2<true, STATS>(S, tr, hu_, tmax, stk, mode, c, lf, st, occ);
                if (fin) {
                    Wv.vis[idx] = occ ? 1 : 0;
                    has = false;
                }
            }
            act = __ballot(has);
            if (act == 0 || (!exhausted && 64 - __popcll(act) >= REFILL)) break;
        }
    }
    if (STATS)
        flush_stats(st, stk, wit, wbusy, &Wv.cnt->sh_node_visits, &Wv.cnt->sh_prim_tests, &Wv.cnt->sh_pruned,
                    &Wv.cnt->sh_iters, &Wv.cnt->sh_lanes_busy, &Wv.cnt->spills);
}

// Host-side launch of the k_shadow instance for (stats, wide records).
static void launch_shadow(bool stats, bool wide, int grid, hipStream_t s, const DevScene& S, const Wave& W, SpillArea sp,
                          bool top = false) {
    const dim3 g(grid), b(TRAV_BLOCK);
    if (top && !stats && !wide && S.top) {
        hipLaunchKernelGGL((k_shadow<false, false, true>), g, b, LDS_BYTES + TOP_LDS_BYTES, s, S, W, sp);
        return;
    }
    if (wide) {
        if (stats) hipLaunchKernelGGL((k_shadow<true, true>), g, b, LDS_BYTES, s, S, W, sp);
        else hipLaunchKernelGGL((k_shadow<false, true>), g, b, LDS_BYTES, s, S, W, sp);
    } else {
        if (stats) hipLaunchKernelGGL((k_shadow<true, false>), g, b, LDS_BYTES, s, S, W, sp);
        else hipLaunchKernelGGL((k_shadow<false, false>), g, b, LDS_BYTES, s, S, W, sp);
    }
}

// ---- path kernel: every bounce of a path in one persistent launch (khp_ctx_params.path_kernel) ----
// KIRK's loop runs every pixel's path to its end, bounce after bounce
// (PathTracer::traceRays, CPU_PathTracer.cpp:129-168).  The wavefront above makes
// each bounce's stages persistent launches, and a launch ends with its slowest
// ray: a synchronous frame pays depth x (extension tail + shadow tail) whatever
// its size -- 11 of the 14.8 ms of a 1-spp 1080p call (profiles/
// r04a_sync_breakdown.md).  k_path carries every path of a chunk through all its
// bounces in ONE persistent launch: a lane traces its path's extension ray,
// shades the hit, traces the shadow ray in the same loop (iter2k<2>: the lane's
// query kind is a per-lane value), adds the colour, continues with the next
// bounce, and claims the next camera path when its path ends.  Only the longest
// path remains a tail.  Shading waits until REFILL lanes of the wave have
// finished their traversals (fewer once every path is claimed), so the shading
// code runs with most lanes active.  A lane's path state (T, C, key, the next
// ray and the deferred NEE terms) lives in global columns (PathLanes, one entry
// per resident lane) while it traverses, so the loop carries traversal
// registers only.  The per-hit arithmetic is k_shade's (the !BD path), the
// any-hit walk k_shadow's and the colour add k_shadow_finish's: frames are
// bit-identical to the wavefront's and the oracle's.
#ifndef KHP_PATH_WAVES
#define KHP_PATH_WAVES 4
#endif
#ifndef KHP_PATH_RING
#define KHP_PATH_RING 8
#endif
#ifndef KHP_PATH_REFILL
#define KHP_PATH_REFILL 24
#endif
constexpr int PATH_WAVES = KHP_PATH_WAVES;
constexpr uint32_t PATH_REFILL = KHP_PATH_REFILL;   // finished lanes that trigger a wave's service
constexpr int PATH_RING = KHP_PATH_RING;
constexpr size_t PATH_LDS_BYTES = 3 * PATH_RING * TRAV_BLOCK * sizeof(uint32_t);

struct PathLanes {
    // [column][grid lane]: 0 T.xyz | flags   1 C.xyz | key   2 next ray o.xyz | path id
    // 3 next ray d.xyz | bounce (bit 31: the path continues after the pending shadow ray)
    // 4 lc.xyz | has_emit   5 Told.xyz   6 AT.xyz   7 ET.xyz  (the deferred NEE terms, k_shade's shadow record)
    float4* col[8];
};

// ---- render-ahead (khp_ctx_params.render_ahead, ABI 13) ---------------------------------------
// KIRK's GUI calls PathTracer::render once per pass and waits for it
// (CPU_PathTracer.cpp:17-52); a synchronous k_path launch ends with the drain
// of its longest paths, ~45% of a 1-spp call with most lanes idle (DESIGN.md
// §5b).  With render-ahead the launch of call k renders the paths of sample
// set k ("own") and, once every own path is claimed, lets its idle lanes claim
// the paths of the sets the NEXT calls of the progressive series will ask for
// (sets k+1 .. k+D: the same pixels, samples first_sample + j*spp ...), set
// after set.  A path that ends writes its colour to its set's column; the
// launch ends as soon as every own path has ended (a counter that the waves
// without an own path poll), and each lane still holding a path of a later set
// parks it: the path state at the start of its current traversal (the 8
// PathLanes columns, the ray, the query kind) is appended to its set's park
// list and the traversal is redone later.  Every launch takes, set by set, the
// parked paths first, then the set's unclaimed paths from the cursors earlier
// launches advanced; call k+1 accumulates the colour column of set k+1.  Paths
// are independent and deterministic functions of (scene, camera, parameters,
// pixel, sample), so each call's colours -- and its accumulate, texture and
// framebuffer -- are those of rendering it alone.  The host drops the sets on
// any change of scene, camera, parameters, size or first_sample (AheadSet).
// The sets live in a ring of nsets = D + 1 slots; a path carries its set
// relative to the launch's own set (0 own, 1 next, ...) in the top bits of its
// PathLanes id.
constexpr uint32_t RA_MAX_SETS = 4;
constexpr uint32_t SET_SHIFT = 30;               // PathLanes col[2].w: bits 30-31 = relative set
constexpr uint32_t PID_MASK = (1u << SET_SHIFT) - 1u;
constexpr uint32_t PARK_F4 = 10;                 // float4 per park record: 8 columns, (o, t_max), (d, any)
struct AheadState;
struct Ahead {
    uint32_t on;         // 0: a plain synchronous launch (the fields below unused)
    uint32_t npaths;     // paths per set (= the launch's own paths)
    uint32_t spp;        // set j's camera paths: sample offset j * spp from the own set's
    uint32_t own;        // ring slot of the own set
    uint32_t nsets;      // sets in flight: the own set and nsets - 1 later ones (2 .. RA_MAX_SETS)
    uint32_t park_cap;   // park records per ring slot
    AheadState* st;
    float4* ck;          // [ring slot][npaths] colour columns (Wave::CK = the own slot's)
    float4* park;        // [ring slot][park_cap][PARK_F4] park lists
};
struct alignas(128) AheadState {
    uint32_t fetch[RA_MAX_SETS][NSEG * 32];   // per ring slot: claim cursors (one 128-B line each)
    uint32_t done[RA_MAX_SETS][32];           // paths of the set that have ended
    uint32_t park_n[RA_MAX_SETS][32];         // records appended to the set's park list
    uint32_t park_lim[RA_MAX_SETS][32];       // park_n when the launch was enqueued: the records it may resume
    uint32_t take[RA_MAX_SETS][32];           // resume cursor over the list
    uint32_t report[32];                      // at enqueue: the own set's finished paths, its resumable records
};
__device__ __forceinline__ uint32_t ra_slot(const Ahead& A, uint32_t j) {
    const uint32_t s = A.own + j;
    return s >= A.nsets ? s - A.nsets : s;
}
// Ends a path: its colour to its set's column; returns 1 + its relative set.
template <bool RA>
__device__ __forceinline__ uint32_t end_path(const Wave& Wv, const Ahead& A, uint32_t pw, float4 cko) {
    const uint32_t j = RA ? pw >> SET_SHIFT : 0u;
    if (RA && j != 0u) {
        A.ck[(size_t)ra_slot(A, j) * A.npaths + (pw & PID_MASK)] = cko;
        return 1u + j;
    }
    Wv.CK[pw & PID_MASK] = cko;
    return 1u;
}
// Every own path of the launch has ended (render-ahead; wave-uniform).
__device__ __forceinline__ bool own_set_done(const Ahead& A) {
    const uint32_t d = __hip_atomic_load(&A.st->done[A.own][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(d) >= A.npaths;
}
// Before a render-ahead launch: clears the ring slots in `clear` (bit mask), then
// fixes every slot's resume limit and the own slot's report.
__global__ void k_ahead_prep(AheadState* a, uint32_t clear, uint32_t own) {
    for (uint32_t p = 0; p < RA_MAX_SETS; ++p) {
        if (!(clear >> p & 1u)) continue;
        for (uint32_t i = threadIdx.x; i < NSEG * 32; i += blockDim.x) a->fetch[p][i] = 0;
        if (threadIdx.x == 0) {
            a->done[p][0] = 0;
            a->park_n[p][0] = 0;
            a->take[p][0] = 0;
        }
    }
    __syncthreads();
    // A resume claim takes a wave's whole request from `take`, also past the limit
    // (those lanes get nothing), so take can end a launch beyond park_lim while the
    // records from park_lim on -- parked by that same launch -- were never resumed:
    // the next launch resumes from park_lim there.
    if (threadIdx.x < RA_MAX_SETS) {
        const uint32_t p = threadIdx.x;
        if (a->take[p][0] > a->park_lim[p][0]) a->take[p][0] = a->park_lim[p][0];
        a->park_lim[p][0] = a->park_n[p][0];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a->report[0] = a->done[own][0];
        a->report[1] = a->park_n[own][0] > a->take[own][0] ? a->park_n[own][0] - a->take[own][0] : 0u;
    }
}

// k_shade's per-hit operations without the light-path variant (KIRK's traceRay
// light test, EnvironmentShader / LightShader / SimpleShader /
// MarschnerHairShader): the path state after bounce `bounce` and, when the NEE
// colour is nonzero, the shadow ray whose any-hit result decides the deferred
// colour add (shadow_finish_one).
struct ShadeOut {
    v3 T, C;
    int flags;
    Ray nr;           // the next extension ray
    bool emit_ray;    // the path continues with nr
    bool emit_sh;     // a shadow ray to trace; the colour add is deferred to its finish
    Ray shr;
    float sh_tmax;
    v3 lc, Told, AT, ET;
    bool has_emit;
};
template <bool TEX, uint32_t KINDS>
__device__ __forceinline__ void shade_core(const DevScene& S, const Ray& r, float lambda, int32_t slot, v3 T, v3 C,
                                           int flags, uint32_t key, uint32_t bounce, bool last, ShadeOut& o) {
    o.nr.o = o.nr.d = mk(0, 0, 0);
    o.shr.o = o.shr.d = mk(0, 0, 0);
    o.sh_tmax = 0.0f;
    o.lc = o.Told = o.AT = o.ET = mk(0, 0, 0);
    o.has_emit = false;
    o.emit_sh = false;
    float t_lights = FLT_MAX_;
    int t_index = -1;
    for (int li = 0; li < S.n_lights; ++li) {
        float t = FLT_MAX_;
        if (light_isect(S.lights[li], r, t)) {
            t_lights = gmin(t_lights, t);
            t_index = (t == t_lights) ? li : t_index;
        }
    }
    bool light_hit = false;
    if (t_lights < lambda) {
        lambda = t_lights;
        light_hit = true;
    }
    if (lambda == FLT_MAX_) {
        C = C + (TEX ? env_color(S, r.d) : mk(S.env.color[0], S.env.color[1], S.env.color[2])) * T;
        T = mk(0, 0, 0);
    } else if (light_hit) {
        C = C + light_emit(S.lights[t_index], r.d) * T;
        T = mk(0, 0, 0);
    } else {
        ShadeCtx s;
        khp_material mres;
        const Hit hh{lambda, slot, 0.0f, 0.0f};
        const v3 nrm = surface_at<TEX>(S, r, hh, s, mres);
        const v3 loc = follow(r, lambda);
        const khp_material* m = s.m;
        float h0 = draw_u01(key, dim_of(bounce, P_HAIR_ALPHA)), h1 = draw_u01(key, dim_of(bounce, P_HAIR_BETA));
        v3 counter = -normalize(r.d);
        bool need_shadow = false;
        if (S.n_lights > 0) {
            int li = (int)((double)draw_u01(key, dim_of(bounce, P_LIGHT_SEL)) * (double)S.n_lights);
            const DevLight& L = S.lights[li];
            float att;
            Ray h2l = light_dir(L, loc, draw_u01(key, dim_of(bounce, P_LIGHT_0)),
                                draw_u01(key, dim_of(bounce, P_LIGHT_1)), att);
            v3 lightpos = h2l.o + h2l.d;
            h2l.o = h2l.o + faceforward(nrm, h2l.o - lightpos, nrm) * 1e-4f;
            h2l.d = normalize(h2l.d);
            if (L.color[0] > 0.0f || L.color[1] > 0.0f || L.color[2] > 0.0f) {
                v3 f = bsdf_eval(s, h2l.d, -r.d);
                float ad = fabsf(dot(h2l.d, nrm));
                o.lc = mk(L.color[0] * ((att * f.x) * ad), L.color[1] * ((att * f.y) * ad),
                          L.color[2] * ((att * f.z) * ad));
                o.sh_tmax = length(lightpos - h2l.o);
                o.shr = h2l;
                need_shadow = true;
            }
        }
        v3 ev = bsdf_eval(s, nrm, nrm);
        v3 amb = mk(S.env.ambient[0], S.env.ambient[1], S.env.ambient[2]) * (ev * ONE_OVER_PI);
        o.Told = T;
        o.AT = amb * T;
        bool add_now = true;
        if (m->shader == KHP_SHADER_MARSCHNER_HAIR) {
            float smp[2] = {0.0f, 0.0f};
            v3 out;
            float pdf = 0.0f;
            bool valid;
            v3 refl = bsdf_sample<KINDS>(s, counter, nrm, smp, h0, h1, out, pdf, flags, valid);
            v3 off = out * 1e-4f;
            if (!(flags & F_SPECULAR)) off = faceforward(-(nrm * 1e-4f), nrm, out);
            o.nr = make_ray(loc + off, out);
            if ((flags & F_CYL_T) || (flags & F_CYL_TR)) {
                need_shadow = false;
                add_now = false;
            } else {
                if (is_zero(refl) || pdf <= 1E-4f || gmax(T.x, gmax(T.y, T.z)) < 0.01f) T = mk(0, 0, 0);
                else T = T * ((refl * 3.0f) * fabsf(k_cosf(smp[0])));
            }
        } else {
            float smp[2] = {draw_u01(key, dim_of(bounce, P_BSDF_0)), draw_u01(key, dim_of(bounce, P_BSDF_1))};
            v3 out;
            float pdf = 0.0f;
            int fl = 0;
            bool valid;
            v3 refl = bsdf_sample<KINDS>(s, counter, nrm, smp, h0, h1, out, pdf, fl, valid);
            if (is_zero(refl) || pdf <= 1E-4f || gmax(T.x, gmax(T.y, T.z)) < 0.01f) {
                T = mk(0, 0, 0);
            } else if ((fl & F_EMISSIVE) == F_EMISSIVE) {
                o.has_emit = true;
                o.ET = mk(m->emission[0], m->emission[1], m->emission[2]) * T;
                T = mk(0, 0, 0);
            } else {
                float ad = fabsf(dot(out, nrm));
                T = T * ((refl * ad) / pdf);
                flags = fl;
                v3 off = out * 1e-4f;
                if ((fl & F_SPECULAR) != F_SPECULAR) off = faceforward(-(nrm * 1e-4f), nrm, out);
                o.nr = make_ray(loc + off, out);
            }
        }
        if (add_now) {
            const v3 lc = o.lc;
            if (need_shadow && !(lc.x == 0.0f && lc.y == 0.0f && lc.z == 0.0f)) {
                o.emit_sh = true;  // the colour add waits for the shadow ray
            } else if (need_shadow) {  // zero light colour: the finish's operations, without the ray (k_shade)
                v3 dl = mk(0, 0, 0) + lc * 1.0f;
                v3 acc = (mk(0, 0, 0) + dl * o.Told) + o.AT;
                if (o.has_emit) acc = acc + o.ET;
                C = C + acc;
            } else {
                v3 acc = (mk(0, 0, 0) + mk(0, 0, 0) * o.Told) + o.AT;
                if (o.has_emit) acc = acc + o.ET;
                C = C + acc;
            }
        }
    }
    o.T = T;
    o.C = C;
    o.flags = flags;
    o.emit_ray = !last && !is_zero(T) && !is_zero(o.nr.d);
}

// shadow_finish_one's colour term for a traced shadow ray.
__device__ __forceinline__ v3 finish_acc(const DevScene& S, const Ray& r, float tmax, bool occ, v3 lc, v3 Told, v3 AT,
                                         bool has_emit, v3 ET) {
    if (!occ) {
        for (int li = 0; li < S.n_lights; ++li) {
            float t;
            if (light_isect(S.lights[li], r, t) && (t < tmax)) {
                occ = true;
                break;
            }
        }
    }
    v3 l = lc * (occ ? 0.0f : 1.0f);
    v3 dl = mk(0, 0, 0) + l;
    v3 acc = (mk(0, 0, 0) + dl * Told) + AT;
    if (has_emit) acc = acc + ET;
    return acc;
}

enum : uint32_t { PS_TRAV = 0u, PS_FIN = 1u, PS_NEW = 2u, PS_BEGIN = 3u, PS_DONE = 4u };

#ifdef KHP_PATH_PROFILE
// Diagnostic builds: one record per k_path wave (100 MHz wall clock): start,
// claim exhaustion seen, end, (traversal-loop iterations << 32 | those after
// exhaustion), traversing lanes summed over the drain iterations, (block << 32 |
// lanes with a path at exhaustion).  Read and reset by khp_debug_wave_profile.
#define KHP_WPROF_MAX 65536
__device__ unsigned long long g_wprof[6 * KHP_WPROF_MAX];
__device__ uint32_t g_wprof_n;
// render-ahead: the clock when the last own path ended, ~ when the first wave saw the own set's end
__device__ unsigned long long g_ra_prof[2];
#endif

// Render-ahead tuning: a wave adds its ended paths to the set counters in batches
// of KHP_RA_BATCH (at once for own paths once the own set is all claimed: the end
// of the set is looked for only then).
#ifndef KHP_RA_BATCH
#define KHP_RA_BATCH 1024
#endif
#ifndef KHP_RA_PROTECT   // only waves without an own path claim later sets' paths
#define KHP_RA_PROTECT 0
#endif
#ifndef KHP_RA_MIX   // measured slower: off
#define KHP_RA_MIX 0
#endif
#ifndef KHP_RA_MIX_REFILL
#define KHP_RA_MIX_REFILL 48
#endif
#ifndef KHP_RA_NO_AHEAD   // diagnostic builds: the render-ahead instance with nothing claimed ahead
#define KHP_RA_NO_AHEAD 0
#endif
// QS (hybrid batches, khp_ctx_params.path_from): the launch takes its paths from the
// wavefront's queue of bounce Wv.q_bounce (parity Wv.q_cur) -- each entry's ray and
// path state (TFq / CKq, moved as k_shade and the shadow finish left them) -- and
// carries them through the remaining bounces; paths of a chunk that ended earlier
// already wrote their colour.
template <bool TEX, bool WIDE, uint32_t KINDS, bool RA, bool QS = false>
__global__ __launch_bounds__(TRAV_BLOCK, PATH_WAVES) void k_path(DevScene S, Wave Wv, SpillArea spill, PathLanes L, Ahead A) {
    extern __shared__ uint32_t lds[];
    const uint32_t npaths = Wv.P * Wv.n_samples * Wv.n_frames;
    const uint32_t g = blockIdx.x * TRAV_BLOCK + threadIdx.x;
    if (RA && own_set_done(A)) return;   // render-ahead: earlier launches finished this whole set
    // render-ahead (wave-uniform): the set the wave claims from (relative: 0 own, 1 the next
    // call's, ...), its resume limit and whether parked records may remain; ended paths per
    // set not yet counted; the lanes holding an own path (only a wave without one looks for
    // the end of the own set: the look is a coherent load, and the waves carrying the call's
    // last paths never wait for it)
    const uint32_t nsets = RA ? (KHP_RA_NO_AHEAD ? 1u : A.nsets) : 1u;
    uint32_t cur = 0u, lim = RA ? __builtin_amdgcn_readfirstlane(A.st->park_lim[A.own][0]) : 0u;
    bool res_left = lim > 0u, stop = false;
    uint32_t pend[RA_MAX_SETS] = {0u, 0u, 0u, 0u}, poll_it = 0u;
    unsigned long long own_lanes = 0ull;
    LdsStack<PATH_RING, false> stk;
    stk.init(lds, spill.base, spill.stride);
    TravStats st{0, 0, 0};
    TravRay tr;
    tr.r.o = tr.r.d = tr.inv = mk(0, 0, 0);
    tr.fin = true;
    Hit h{FLT_MAX_, -1, 0.0f, 0.0f};
    Cur c{0u, 0.0f, 0.0f, false};
    LeafCur lf{0u, 0u, 0.0f, 0.0f, 0.0f, 0.0f, -1};
    uint32_t mode = 0u, state = PS_NEW, n_ext = 0, n_sh = 0;
    bool any = false, occ = false, exhausted = false;
    float tmax_any = 0.0f;
    Claimer cl;   // the claims of set `cur` (render-ahead), of the launch's paths otherwise
    if (QS) cl.init(Wv.cnt->fetch_ext, Wv.cnt->nq[Wv.q_cur], Wv.cnt->nqb[Wv.q_cur], Wv.cap);
    else cl.init(RA ? A.st->fetch[A.own] : Wv.cnt->fetch_ext, npaths, 0u, npaths);
#ifdef KHP_PATH_PROFILE   // diagnostic builds: launch timeline (100 MHz wall clock): first start, last
    // claim exhaustion seen, last end, longest drain of one wave (its end - its exhaustion)
    const unsigned long long pc_start = wall_clock64();
    unsigned long long pc_exh = 0;
    uint32_t pw_iters = 0, pw_drain_iters = 0, pw_ntrav_exh = 0;   // per-wave record (g_wprof)
    unsigned long long pw_drain_lanes = 0;
#endif
    for (;;) {
#ifdef KHP_PATH_PROFILE
        if ((RA ? cur > 0u : exhausted) && pc_exh == 0) {
            pc_exh = wall_clock64();
            pw_ntrav_exh = (uint32_t)__popcll(__ballot(state == PS_TRAV || state == PS_FIN || state == PS_BEGIN));
        }
#endif
        // render-ahead: once every own path has ended, park the later sets' paths (below) and leave
        if (RA && (stop || (cur > 0u && own_lanes == 0ull && own_set_done(A)))) {
#ifdef KHP_PATH_PROFILE
            if (lane_id() == 0) atomicMin(&g_ra_prof[1], wall_clock64());
#endif
            stop = true;
            break;
        }
        // ---- service: shade finished extension rays, finish shadow rays, claim camera
        //      paths, start traversals -- until every lane traverses or has no work left
        for (;;) {
            Ray sray;          // the ray a lane starts next (PS_BEGIN)
            bool sany = false;
            float stmax = 0.0f;
            uint32_t ended = 0u;   // render-ahead: 1 + the relative set of a path that ended here
            bool st_own = false;   // render-ahead: an own path started here
            sray.o = sray.d = mk(0, 0, 0);
            if (state == PS_FIN) {
                const Ray fr = tr.r;
                if (!any) {  // k_shade
                    const float4 f0 = L.col[0][g], f1 = L.col[1][g], f2 = L.col[2][g], f3 = L.col[3][g];
                    const uint32_t bounce = bits_from_f(f3.w) & 0xFFFFu;
                    ShadeOut o;
                    shade_core<TEX, KINDS>(S, fr, h.t, h.slot, mk(f0.x, f0.y, f0.z), mk(f1.x, f1.y, f1.z),
                                           (int)bits_from_f(f0.w), bits_from_f(f1.w), bounce, bounce + 1 >= Wv.depth, o);
                    ++n_ext;
                    const float4 tfo = make_float4(o.T.x, o.T.y, o.T.z, f_from_bits((uint32_t)o.flags));
                    const float4 cko = make_float4(o.C.x, o.C.y, o.C.z, f1.w);
                    if (o.emit_sh) {
                        L.col[0][g] = tfo;
                        L.col[1][g] = cko;
                        L.col[2][g] = make_float4(o.nr.o.x, o.nr.o.y, o.nr.o.z, f2.w);
                        L.col[3][g] = make_float4(o.nr.d.x, o.nr.d.y, o.nr.d.z,
                                                  f_from_bits(bounce | (o.emit_ray ? 0x80000000u : 0u)));
                        L.col[4][g] = make_float4(o.lc.x, o.lc.y, o.lc.z, o.has_emit ? 1.0f : 0.0f);
                        L.col[5][g] = make_float4(o.Told.x, o.Told.y, o.Told.z, 0.0f);
                        L.col[6][g] = make_float4(o.AT.x, o.AT.y, o.AT.z, 0.0f);
                        L.col[7][g] = make_float4(o.ET.x, o.ET.y, o.ET.z, 0.0f);
                        sray = o.shr;
                        stmax = o.sh_tmax;
                        sany = true;
                        state = PS_BEGIN;
                    } else if (o.emit_ray) {
                        L.col[0][g] = tfo;
                        L.col[1][g] = cko;
                        L.col[3][g] = make_float4(0.0f, 0.0f, 0.0f, f_from_bits(bounce + 1u));
                        sray = o.nr;
                        state = PS_BEGIN;
                    } else {
                        ended = end_path<RA>(Wv, A, bits_from_f(f2.w), cko);
                        state = PS_NEW;
                    }
                } else {  // k_shadow_finish
                    const float4 f1 = L.col[1][g], f2 = L.col[2][g], f3 = L.col[3][g], f4 = L.col[4][g];
                    const float4 f5 = L.col[5][g], f6 = L.col[6][g], f7 = L.col[7][g];
                    const v3 acc = finish_acc(S, fr, tmax_any, occ, mk(f4.x, f4.y, f4.z), mk(f5.x, f5.y, f5.z),
                                              mk(f6.x, f6.y, f6.z), f4.w != 0.0f, mk(f7.x, f7.y, f7.z));
                    ++n_sh;
                    const float4 cko = make_float4(f1.x + acc.x, f1.y + acc.y, f1.z + acc.z, f1.w);
                    const uint32_t b3 = bits_from_f(f3.w);
                    if (b3 & 0x80000000u) {
                        L.col[1][g] = cko;
                        L.col[3][g] = make_float4(0.0f, 0.0f, 0.0f, f_from_bits((b3 & 0xFFFFu) + 1u));
                        sray.o = mk(f2.x, f2.y, f2.z);
                        sray.d = mk(f3.x, f3.y, f3.z);
                        state = PS_BEGIN;
                    } else {
                        ended = end_path<RA>(Wv, A, bits_from_f(f2.w), cko);
                        state = PS_NEW;
                    }
                }
            }
            if (RA) {   // render-ahead: ended paths per set
                const unsigned long long eom = __ballot(ended == 1u);
                pend[0] += (uint32_t)__popcll(eom);
                for (uint32_t j = 1; j < RA_MAX_SETS; ++j) pend[j] += (uint32_t)__popcll(__ballot(ended == 1u + j));
                own_lanes &= ~eom;
                // KHP_RA_PROTECT: a wave that idled lanes while it carried own paths takes
                // later sets' paths again once they have all ended
                if (KHP_RA_PROTECT && own_lanes == 0ull && cur > 0u && cur < nsets && state == PS_DONE) state = PS_NEW;
#ifdef KHP_PATH_PROFILE
                if (eom && lane_id() == 0) atomicMax(&g_ra_prof[0], wall_clock64());
#endif
            }
            unsigned long long want = __ballot(state == PS_NEW);
            if (want != 0ull) {  // wave-uniform: claim paths for the lanes whose path ended
                bool cam = false;   // a camera path starts: path cpid (with its relative set), sample offset coff
                uint32_t cpid = 0, coff = 0;
                if constexpr (RA) {
                    // set after set (own first): its parked paths, then its unclaimed ones
                    while (want != 0ull && cur < nsets &&
                           !(KHP_RA_PROTECT && cur > 0u && (own_lanes | __ballot(st_own)) != 0ull)) {
                        const uint32_t sl = ra_slot(A, cur);
                        if (res_left) {
                            const uint32_t slot = wave_alloc(state == PS_NEW && !cam, &A.st->take[sl][0]);
                            if (__ballot(state == PS_NEW && !cam && slot >= lim) != 0ull) res_left = false;
                            if (state == PS_NEW && !cam && slot < lim) {
                                const float4* r = A.park + ((size_t)sl * A.park_cap + slot) * PARK_F4;
#pragma unroll 1
                                for (int k = 0; k < 8; ++k) {   // one record at a time (registers)
                                    float4 v = r[k];
                                    if (k == 2) v.w = f_from_bits((bits_from_f(v.w) & PID_MASK) | (cur << SET_SHIFT));
                                    L.col[k][g] = v;
                                }
                                const float4 ro = r[8], rd = r[9];
                                sray.o = mk(ro.x, ro.y, ro.z);
                                sray.d = mk(rd.x, rd.y, rd.z);
                                stmax = ro.w;
                                sany = bits_from_f(rd.w) != 0u;
                                state = PS_BEGIN;
                                st_own = cur == 0u;
                            }
                        } else if (!exhausted) {
                            uint32_t my = 0, pid = 0;
                            const bool got = cl.claim(want, my, exhausted);
                            if (state == PS_NEW && !cam && got && cl.phys(my, pid)) {
                                cam = true;
                                cpid = pid | (cur << SET_SHIFT);
                                coff = cur * A.spp;
                                st_own = cur == 0u;
                            }
                        } else if (++cur < nsets) {   // the next set: its cursors and park list
                            const uint32_t s2 = ra_slot(A, cur);
                            cl.retarget(A.st->fetch[s2]);
                            exhausted = false;
                            lim = __builtin_amdgcn_readfirstlane(A.st->park_lim[s2][0]);
                            res_left = lim > 0u;
                        }
                        want = __ballot(state == PS_NEW && !cam);
                    }
                    own_lanes |= __ballot(st_own);
                    if (state == PS_NEW && (cur >= nsets || (KHP_RA_PROTECT && cur > 0u && own_lanes != 0ull)))
                        state = PS_DONE;
                } else if constexpr (QS) {   // the next queue entry: its ray and path state
                    uint32_t my = 0, slot = 0;
                    bool got = false;
                    if (!exhausted) got = cl.claim(want, my, exhausted);
                    if (state == PS_NEW && got && cl.phys(my, slot)) {
                        const uint32_t qc = Wv.q_cur;
                        const uint32_t src = Wv.qsrc ? Wv.qsrc[slot] : slot;   // regrouped rays: state slot
                        L.col[0][g] = Wv.TFq[qc][src];
                        L.col[1][g] = Wv.CKq[qc][src];
                        L.col[2][g] = make_float4(0.0f, 0.0f, 0.0f, f_from_bits(Wv.qpid[qc][slot]));
                        L.col[3][g] = make_float4(0.0f, 0.0f, 0.0f, f_from_bits(Wv.q_bounce));
                        sray.o = mk(Wv.qo[qc][0][slot], Wv.qo[qc][1][slot], Wv.qo[qc][2][slot]);
                        sray.d = mk(Wv.qd[qc][0][slot], Wv.qd[qc][1][slot], Wv.qd[qc][2][slot]);
                        sany = false;
                        state = PS_BEGIN;
                    }
                } else {
                    uint32_t my = 0, pid = 0;
                    bool got = false;
                    if (!exhausted) got = cl.claim(want, my, exhausted);
                    if (state == PS_NEW && got && cl.phys(my, pid)) {
                        cam = true;
                        cpid = pid;
                    }
                }
                if (cam) {
                    uint32_t key;
                    sray = camera_path(S, Wv, cpid & PID_MASK, key, coff);
                    L.col[0][g] = make_float4(1.0f, 1.0f, 1.0f, f_from_bits(0u));
                    L.col[1][g] = make_float4(0.0f, 0.0f, 0.0f, f_from_bits(key));
                    L.col[2][g] = make_float4(0.0f, 0.0f, 0.0f, f_from_bits(cpid));
                    L.col[3][g] = make_float4(0.0f, 0.0f, 0.0f, f_from_bits(0u));
                    sany = false;
                    state = PS_BEGIN;
                }
                if (!RA && state == PS_NEW && exhausted) state = PS_DONE;
            }
            if (RA) {   // render-ahead: add the ended paths to their sets' counters
                if (pend[0] != 0u && (cur > 0u || pend[0] >= KHP_RA_BATCH)) {
                    if (lane_id() == 0) atomicAdd(&A.st->done[A.own][0], pend[0]);
                    pend[0] = 0u;
                }
                for (uint32_t j = 1; j < RA_MAX_SETS; ++j) {
                    if (pend[j] >= KHP_RA_BATCH) {
                        if (lane_id() == 0) atomicAdd(&A.st->done[ra_slot(A, j)][0], pend[j]);
                        pend[j] = 0u;
                    }
                }
            }
            if (state == PS_BEGIN) {  // k_extend's / k_shadow's ray start
                TravRay t2;
                trav_setup(t2, sray);
                Hit h2{FLT_MAX_, -1, 0.0f, 0.0f};
                Cur c2{0u, 0.0f, 0.0f, false};
                LeafCur l2{0u, 0u, 0.0f, 0.0f, 0.0f, 0.0f, -1};
                uint32_t m2 = 0u;
                bool o2 = false, go;
                if (!sany) {  // a NaN extension ray: no hit
                    go = !ray_has_nan(sray) && trav2_begin<false>(S, t2, h2.t, stk, m2, c2, l2, st);
                } else if (x_slab_nan(t2)) {
                    o2 = any_hit_x_nan(S, sray);
                    go = false;
                } else {
                    go = trav2_begin<false>(S, t2, stmax, stk, m2, c2, l2, st);
                }
                state = go ? PS_TRAV : PS_FIN;
                tr = t2;
                h = h2;
                c = c2;
                lf = l2;
                mode = m2;
                any = sany;
                occ = o2;
                tmax_any = stmax;
            }
            if (__ballot(state == PS_FIN || state == PS_BEGIN || state == PS_NEW) == 0ull) break;
        }
        if (__ballot(state == PS_TRAV) == 0ull) break;  // every lane done: no path left
        // ---- traversal: one record per lane per iteration, closest or any hit per lane
        for (;;) {
            if (state == PS_TRAV) {
                bool o2 = false;
                const bool f = WIDE ? iterwk<2, false>(S, tr, h, tmax_any, stk, mode, c, lf, st, o2, any)
                                    : iter2k<2, false>(S, tr, h, tmax_any, stk, mode, c, lf, st, o2, any);
                if (f) {
                    state = PS_FIN;
                    occ = o2;
                }
            }
            const uint32_t ntrav = (uint32_t)__popcll(__ballot(state == PS_TRAV));
            const uint32_t nfin = (uint32_t)__popcll(__ballot(state == PS_FIN));
#ifdef KHP_PATH_PROFILE
            ++pw_iters;
            if (pc_exh != 0) {
                ++pw_drain_iters;
                pw_drain_lanes += ntrav;
            }
#endif
            // refill at REFILL finished lanes; once every path is claimed, as soon as
            // the finished lanes are as many as those still traversing (the drain;
            // servicing at every finished lane there measured 5% slower)
            const bool nomore = RA ? (cur >= nsets || (KHP_RA_PROTECT && cur > 0u && own_lanes != 0ull)) : exhausted;
            uint32_t thr = nomore ? (ntrav < PATH_REFILL ? (ntrav > 0u ? ntrav : 1u) : PATH_REFILL) : PATH_REFILL;
            if (RA && KHP_RA_MIX && cur > 0u && own_lanes != 0ull) {
                // render-ahead, a wave carrying own paths beside later sets' ones once the own set is
                // claimed: an own path that finished its traversal is shaded at once (the call waits
                // for it), the others wait for KHP_RA_MIX_REFILL finished lanes
                if (__ballot(state == PS_FIN) & own_lanes) break;
                thr = nomore ? thr : KHP_RA_MIX_REFILL;
            }
            if (ntrav == 0u || nfin >= thr) break;
            // render-ahead: a wave busy with later sets' paths looks for the end of the own set
            // every 32 iterations too (its lanes may not finish a traversal for long)
            if (RA && cur > 0u && own_lanes == 0ull && (++poll_it & 31u) == 0u && own_set_done(A)) {
                stop = true;
                break;
            }
        }
    }
    if (RA) {   // render-ahead: the counts not yet added
        for (uint32_t j = 0; j < RA_MAX_SETS; ++j)
            if (pend[j] != 0u && lane_id() == 0) atomicAdd(&A.st->done[ra_slot(A, j)][0], pend[j]);
    }
    if (RA && stop) {   // render-ahead: later sets' paths are appended to their park lists, each as
                        // its state at the start of its current traversal, which is redone
        uint32_t j = 0u;
        if (state == PS_TRAV || state == PS_FIN) j = bits_from_f(L.col[2][g].w) >> SET_SHIFT;
        for (uint32_t q = 1; q < nsets; ++q) {
            const uint32_t sl = ra_slot(A, q);
            const uint32_t slot = wave_alloc(j == q, &A.st->park_n[sl][0]);
            if (j == q && slot < A.park_cap) {   // (park_cap holds every lane of nsets - 1 launches)
                float4* r = A.park + ((size_t)sl * A.park_cap + slot) * PARK_F4;
                for (int k = 0; k < 8; ++k) r[k] = L.col[k][g];
                r[8] = make_float4(tr.r.o.x, tr.r.o.y, tr.r.o.z, tmax_any);
                r[9] = make_float4(tr.r.d.x, tr.r.d.y, tr.r.d.z, f_from_bits(any ? 1u : 0u));
            }
        }
    }
    const unsigned long long se = wave_sum((unsigned long long)n_ext), ss = wave_sum((unsigned long long)n_sh);
    if (lane_id() == 0) {
        atomicAdd(&Wv.cnt->ext_rays, se);
        atomicAdd(&Wv.cnt->sh_rays, ss);
#ifdef KHP_PATH_PROFILE
        const unsigned long long pc_end = wall_clock64();
        if (pc_exh == 0) pc_exh = pc_end;
        atomicMax(&Wv.cnt->step_cycles[0], ~pc_start);
        atomicMax(&Wv.cnt->step_cycles[1], pc_exh);
        atomicMax(&Wv.cnt->step_cycles[2], pc_end);
        atomicMax(&Wv.cnt->step_cycles[3], pc_end - pc_exh);
        const uint32_t slot = atomicAdd(&g_wprof_n, 1u);
        if (slot < KHP_WPROF_MAX) {
            unsigned long long* r = g_wprof + 6 * (size_t)slot;
            r[0] = pc_start;
            r[1] = pc_exh;
            r[2] = pc_end;
            r[3] = ((unsigned long long)pw_iters << 32) | pw_drain_iters;
            r[4] = pw_drain_lanes;
            r[5] = ((unsigned long long)blockIdx.x << 32) | pw_ntrav_exh;
        }
#endif
    }
}

constexpr size_t PATH_LDS = PATH_LDS_BYTES;
// BSDF kind sets k_path is instantiated for: every kind, or the fur scenes'
// (Lambert reflection + Marschner hair: configs 1-3 and the metric row), where
// the other kinds' code and registers are compiled out.
constexpr uint32_t KINDS_ALL = (1u << KHP_BSDF_COUNT) - 1u;
constexpr uint32_t KINDS_FUR = (1u << KHP_BSDF_LAMBERTIAN_REFLECTION) | (1u << KHP_BSDF_MARSCHNER_HAIR);
template <bool TEX, bool WIDE, uint32_t K>
static void launch_path_k(int grid, hipStream_t s, const DevScene& S, const Wave& W, SpillArea sp, const PathLanes& L,
                          const Ahead& A, bool qs) {
    if (qs) {
        hipLaunchKernelGGL((k_path<TEX, WIDE, K, false, true>), dim3(grid), dim3(TRAV_BLOCK), PATH_LDS, s, S, W, sp, L, A);
        return;
    }
    if (A.on) hipLaunchKernelGGL((k_path<TEX, WIDE, K, true>), dim3(grid), dim3(TRAV_BLOCK), PATH_LDS, s, S, W, sp, L, A);
    else hipLaunchKernelGGL((k_path<TEX, WIDE, K, false>), dim3(grid), dim3(TRAV_BLOCK), PATH_LDS, s, S, W, sp, L, A);
}
static void launch_path(bool tex, bool wide, bool fur, int grid, hipStream_t s, const DevScene& S, const Wave& W,
                        SpillArea sp, const PathLanes& L, const Ahead& A, bool qs = false) {
    if (tex) {
        if (wide) launch_path_k<true, true, KINDS_ALL>(grid, s, S, W, sp, L, A, qs);
        else launch_path_k<true, false, KINDS_ALL>(grid, s, S, W, sp, L, A, qs);
    } else if (fur) {
        if (wide) launch_path_k<false, true, KINDS_FUR>(grid, s, S, W, sp, L, A, qs);
        else launch_path_k<false, false, KINDS_FUR>(grid, s, S, W, sp, L, A, qs);
    } else {
        if (wide) launch_path_k<false, true, KINDS_ALL>(grid, s, S, W, sp, L, A, qs);
        else launch_path_k<false, false, KINDS_ALL>(grid, s, S, W, sp, L, A, qs);
    }
}

// ---- accumulate: PathTracer::drawTexture running mean (CPU_PathTracer.cpp:61-90) -------

// Fused frames are accumulated one frame per launch (fr), in call order.
__global__ __launch_bounds__(256) void k_accumulate(Wave Wv, float* fb, uint32_t fr) {
    uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= Wv.P) return;
    uint32_t pixel = Wv.pix[Wv.p_off + p];
    float* o = fb + 3 * (size_t)pixel;
    float r = o[0], g = o[1], b = o[2];
    const size_t base = path_index(Wv, fr, p, 0);
    for (uint32_t s = 0; s < Wv.n_samples; ++s) {
        const float4 ck = Wv.CK[base + s];
        float cr = ck.x, cg = ck.y, cb = ck.z;
        uint32_t k = Wv.fsample0[fr] + s;
        if (k == 0) {
            r = cr; g = cg; b = cb;
        } else {
            float kk = (float)(k + 1);
            r = r + (cr - r) / kk;
            g = g + (cg - g) / kk;
            b = b + (cb - b) / kk;
        }
    }
    o[0] = r; o[1] = g; o[2] = b;
}

// All fused frames of a chunk in one launch (a batch with no gather or snapshot
// between its frames): the same running mean, frame after frame in call order,
// with one framebuffer read and write per pixel instead of one per frame.  A
// block of ACC_PIX pixels stages each frame's samples through LDS: the block
// reads them as whole 16-B-per-lane runs of consecutive samples (a pixel's
// n_samples colours of one frame are adjacent paths), then every thread folds
// its own pixel's samples in order.  Reading them lane-per-pixel instead, 4 KB
// apart with 32 fused frames, fetched 5.6x the bytes (rocprofv3, round 3).
constexpr uint32_t ACC_PIX = 128;
constexpr uint32_t ACC_MAX_SAMPLES = 16;  // LDS: ACC_PIX x (n_samples + 1) float4
__global__ __launch_bounds__(ACC_PIX) void k_accumulate_all(Wave Wv, float* fb) {
    extern __shared__ float4 stage[];
    const uint32_t ns = Wv.n_samples, row = ns + 1u;  // +1: rows start on different banks
    const uint32_t p0 = blockIdx.x * ACC_PIX, np = min(ACC_PIX, Wv.P - p0);
    const uint32_t p = p0 + threadIdx.x;
    float r = 0.0f, g = 0.0f, b = 0.0f;
    float* o = nullptr;
    if (threadIdx.x < np) {
        o = fb + 3 * (size_t)Wv.pix[Wv.p_off + p];
        r = o[0]; g = o[1]; b = o[2];
    }
    for (uint32_t fr = 0; fr < Wv.n_frames; ++fr) {
        for (uint32_t j = threadIdx.x; j < np * ns; j += ACC_PIX) {
            const uint32_t q = j / ns, s = j - q * ns;
            stage[q * row + s] = Wv.CK[path_index(Wv, fr, p0 + q, s)];
        }
        __syncthreads();
        if (threadIdx.x < np) {
            for (uint32_t s = 0; s < ns; ++s) {
                const float4 ck = stage[threadIdx.x * row + s];
                const uint32_t k = Wv.fsample0[fr] + s;
                if (k == 0) {
                    r = ck.x; g = ck.y; b = ck.z;
                } else {
                    const float kk = (float)(k + 1);
                    r = r + (ck.x - r) / kk;
                    g = g + (ck.y - g) / kk;
                    b = b + (ck.z - b) / kk;
                }
            }
        }
        __syncthreads();
    }
    if (o) { o[0] = r; o[1] = g; o[2] = b; }
}

// ---- output stage: Texture::setPixel byte conversion and Tonemapper::map ---------------
// Texture::toByte (Texture.h:252-254): (uchar)std::max(std::min(f * 255, 255), 0).
// std::min(a, b) = (b < a) ? b : a and std::max(a, b) = (a < b) ? b : a, so a
// NaN passes both and its conversion is undefined in C++; x86 and gfx950 both
// give 0, which is the value used here.
__device__ __forceinline__ uint8_t to_byte(float f) {
    const float a = f * 255.0f;
    const float lo = (255.0f < a) ? 255.0f : a;
    const float v = (lo < 0.0f) ? 0.0f : lo;
    return (v == v) ? (uint8_t)(uint32_t)v : (uint8_t)0;
}

__global__ void k_rgba8(const float* fb, uint32_t n, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* c = fb + 3 * (size_t)i;
    uchar4 o = make_uchar4(to_byte(c[0]), to_byte(c[1]), to_byte(c[2]), 255);
    reinterpret_cast<uchar4*>(out)[i] = o;
}

// Tonemapper::RGB_to_Yxy (Tonemapping.cpp:66-91): per pixel Yxy, the max
// luminance (glm::max, NaN-ignoring: order-independent, reduced per block) and
// the pixel's log-luminance term log(2.3e-5 + Y) (k_log_d, the documented
// replacement of the CRT log).  KIRK's sum of those terms is a sequential
// float running sum (`float sum; sum += log(...)`), which no reordering
// reproduces, so the host adds the terms in pixel order.
__device__ __forceinline__ float gdot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    return (a0 * b0 + a1 * b1) + a2 * b2;  // glm::dot operand order
}
__global__ __launch_bounds__(256) void k_tm_yxy(const float* fb, uint32_t n, float* yxy, float* bmax, double* lgv) {
    __shared__ float smax[256];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    float Y = 0.0f, xx = 0.0f, yy = 0.0f, mx = 1e-06f;
    double lg = 0.0;
    if (i < n) {
        const float r = fb[3 * (size_t)i], g = fb[3 * (size_t)i + 1], b = fb[3 * (size_t)i + 2];
        const float X = gdot3(0.5141364f, 0.3238786f, 0.16036376f, r, g, b);
        const float Yv = gdot3(0.265068f, 0.67023428f, 0.06409157f, r, g, b);
        const float Z = gdot3(0.0241188f, 0.1228178f, 0.84442666f, r, g, b);
        const float W = gdot3(X, Yv, Z, 1.0f, 1.0f, 1.0f);
        if (W > 0.0f) {
            Y = Yv;
            xx = X / W;
            yy = Yv / W;
        }
        mx = (mx < Y) ? Y : mx;
        lg = k_log_d(2.3e-5 + (double)Y);
        lgv[i] = lg;
        yxy[3 * (size_t)i] = Y;
        yxy[3 * (size_t)i + 1] = xx;
        yxy[3 * (size_t)i + 2] = yy;
    }
    (void)lg;
    smax[threadIdx.x] = mx;
    __syncthreads();
    for (uint32_t w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const float o = smax[threadIdx.x + w];
            smax[threadIdx.x] = (smax[threadIdx.x] < o) ? o : smax[threadIdx.x];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) bmax[blockIdx.x] = smax[0];
}

// Tonemapper::luminance_from_center (Tonemapping.cpp:183-245): the log terms
// of the Gaussian-weighted window, with the reference's i1 = x*(y_start+ks)+y
// indexing, in KIRK's loop order (t = i * ks + j); the host adds them in that
// order (a sequential double sum).  mask (ks*ks doubles) and `mean` are built
// on the host.
__global__ __launch_bounds__(256) void k_tm_center(const float* yxy, int ks, int xs, int ys, const double* mask,
                                                   double mean, double* terms) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < ks * ks) {
        const int i = t / ks, j = t % ks;
        const int i1 = (xs + i) * (ys + ks) + (ys + j);
        terms[t] = k_log_d(2.3e-5 + (double)yxy[3 * (size_t)i1] * mask[j * ks + i] * mean);
    }
}

struct TmScalars {
    float av_lum, biasP, contP, Lmax, divider, exposure, inv_gamma, slope, start, white, black;
    int contrast_on, gamma_on, rec, clamp_on;
};

// Tonemapper::tonemapping + Yxy_to_RGB + gamma_calc / rec_gamma_calc + clamp,
// then Texture::setPixel(vec4(rgb, 1)).
__global__ __launch_bounds__(256) void k_tm_map(const float* yxy, uint32_t n, TmScalars t, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = yxy[3 * (size_t)i];
    const float xc = yxy[3 * (size_t)i + 1], yc = yxy[3 * (size_t)i + 2];
    if (t.contrast_on) v = k_powf_d(v, t.contP);
    v /= t.av_lum;
    v *= t.exposure;
    const float bias = (float)k_pow_d((double)(v / t.Lmax), (double)t.biasP);
    const float interpol = k_logf_d(2.0f + bias * 8.0f);
    v = k_logf_d(v + 1.0f) / interpol / t.divider;
    const float eps = 1e-06f;
    float X, Z;
    if (v > eps && xc > eps && yc > eps) {
        X = xc * v / yc;
        Z = X / xc - X - v;
    } else {
        X = Z = eps;
    }
    float rgb[3] = {gdot3(2.5651f, -1.1665f, -0.3986f, X, v, Z), gdot3(-1.0217f, 1.9777f, 0.0439f, X, v, Z),
                    gdot3(0.0753f, -0.2543f, 1.1892f, X, v, Z)};
    for (int k = 0; k < 3; ++k) {
        float c = rgb[k];
        if (t.gamma_on) {
            if (t.rec) c = c <= t.start ? c * t.slope : (float)(1.099 * (double)k_powf_d(c, t.inv_gamma) - 0.099);
            else c = k_powf_d(c, t.inv_gamma);
        }
        if (t.clamp_on) {
            c = (c < t.black) ? t.black : c;  // glm::clamp = min(max(x, lo), hi)
            c = (t.white < c) ? t.white : c;
        }
        rgb[k] = c;
    }
    reinterpret_cast<uchar4*>(out)[i] = make_uchar4(to_byte(rgb[0]), to_byte(rgb[1]), to_byte(rgb[2]), 255);
}

// ---- batch ray queries for khp_trace_* ---------------------------------------------------
template <bool STATS>
__global__ __launch_bounds__(256) void k_trace_closest(DevScene S, uint32_t n, const float* orig, const float* dir,
                                                       float* t_out, int32_t* obj_out, float* uv_out,
                                                       unsigned long long* stats) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    TravStats st{0, 0};
    if (i < n) {
        Ray r = make_ray(ld3(orig + 3 * (size_t)i), ld3(dir + 3 * (size_t)i));
        Hit h;
        PrivStack stk;
        trace_closest<STATS>(S, r, h, stk, st);
        t_out[i] = h.t;
        obj_out[i] = h.slot >= 0 ? (int32_t)S.aux[h.slot].obj : -1;
        if (uv_out) {
            uv_out[2 * (size_t)i] = h.u;
            uv_out[2 * (size_t)i + 1] = h.v;
        }
    }
    if (STATS) {
        unsigned long long a = wave_sum((unsigned long long)st.nodes), b = wave_sum((unsigned long long)st.prims);
        if (lane_id() == 0) {
            atomicAdd(&stats[0], a);
            atomicAdd(&stats[1], b);
        }
    }
}

__global__ __launch_bounds__(256) void k_trace_any(DevScene S, uint32_t n, const float* orig, const float* dir,
                                                   const float* tmax, uint8_t* hit_out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Ray r = make_ray(ld3(orig + 3 * (size_t)i), ld3(dir + 3 * (size_t)i));
    TravStats st{0, 0};
    PrivStack stk;
    hit_out[i] = trace_any<false>(S, r, tmax[i], stk, st) ? 1 : 0;
}

// The slot of every triangle (object-id order) for any_hit_x_nan.  Pad slots are zero records.
__global__ void k_tri_slots(const float4* prims, const Aux* aux, uint32_t n_slots, uint32_t n_tris, uint32_t* out) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots || !is_tri(prims[4 * (size_t)s])) return;
    const uint32_t o = aux[s].obj;
    if (o < n_tris) out[o] = s;
}

// Two-level records (traverse.h iterw) from the 64-B node records, one thread
// per record.  Sets *bad when an interior child's box is not the std::min /
// std::max union of its children's boxes, or a child box of it is not ordered
// (mn <= mx on every axis, NaN fails): the composition in iterw would not be
// KIRK's slab then, and the context keeps the 64-B loop.
// The tree's top three levels of interior nodes in BFS order, for the instances
// that stage them in LDS (khp_ctx_params.lds_nodes): the refs between them
// rewritten to TOP_REF | index; everything else (boxes, leaf and deeper refs,
// counts) as in the node array, so the walk, its order and its counts are KIRK's.
__global__ void k_top_nodes(const DevNode* __restrict__ nodes, int32_t root_ref, DevNode* __restrict__ top) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    uint32_t ids[TOP_NODES], depth[TOP_NODES], n = 0;
    if (((uint32_t)root_ref & LEAF_BIT) == 0u) {
        ids[n] = (uint32_t)root_ref;
        depth[n++] = 0;
    }
    for (uint32_t k = 0; k < n; ++k)
        for (int ch = 0; ch < 2; ++ch) {
            const uint32_t r = (uint32_t)nodes[ids[k]].ref[ch];
            if ((r & LEAF_BIT) == 0u && depth[k] + 1u < 3u && n < TOP_NODES) {
                ids[n] = r;
                depth[n++] = depth[k] + 1u;
            }
        }
    for (uint32_t k = 0; k < TOP_NODES; ++k) {
        DevNode o{};
        if (k < n) {
            o = nodes[ids[k]];
            for (int ch = 0; ch < 2; ++ch)
                for (uint32_t j = 1; j < n; ++j)
                    if ((uint32_t)o.ref[ch] == ids[j]) o.ref[ch] = (int32_t)(TOP_REF | j);
        }
        top[k] = o;
    }
}

__global__ void k_wide_records(const DevNode* nodes, uint32_t n, float4* wide, uint32_t* bad) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const DevNode X = nodes[r];
    const bool pad = X.ref[0] == 0 && X.ref[1] == 0;  // unused record of a pair (no node has the root as child)
    float4 o[6];
    int32_t gref[4] = {0, 0, 0, 0};
    bool ok = true;
    for (int k = 0; k < 2; ++k) {
        const uint32_t cr = (uint32_t)X.ref[k];
        // C's box as stored in X (left: a0 a1 a2 | a3 b0 b1; right: b2 b3 c0 | c1 c2 c3)
        const float cb[6] = {k ? X.b[2] : X.a[0], k ? X.b[3] : X.a[1], k ? X.c[0] : X.a[2],
                             k ? X.c[1] : X.a[3], k ? X.c[2] : X.b[0], k ? X.c[3] : X.b[1]};
        if (pad || (cr & LEAF_BIT)) {
            o[3 * k] = make_float4(cb[0], cb[1], cb[2], cb[3]);
            o[3 * k + 1] = make_float4(cb[4], cb[5], 0.0f, 0.0f);
            o[3 * k + 2] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            continue;
        }
        const DevNode C = nodes[cr];
        o[3 * k] = make_float4(C.a[0], C.a[1], C.a[2], C.a[3]);
        o[3 * k + 1] = make_float4(C.b[0], C.b[1], C.b[2], C.b[3]);
        o[3 * k + 2] = make_float4(C.c[0], C.c[1], C.c[2], C.c[3]);
        gref[2 * k] = C.ref[0];
        gref[2 * k + 1] = C.ref[1];
        const float l[6] = {C.a[0], C.a[1], C.a[2], C.a[3], C.b[0], C.b[1]};
        const float rr[6] = {C.b[2], C.b[3], C.c[0], C.c[1], C.c[2], C.c[3]};
        for (int a = 0; a < 3; ++a) {
            ok = ok && l[a] <= l[a + 3] && rr[a] <= rr[a + 3];
            ok = ok && __float_as_uint(wmin(l[a], rr[a])) == __float_as_uint(cb[a]);
            ok = ok && __float_as_uint(wmax(l[a + 3], rr[a + 3])) == __float_as_uint(cb[a + 3]);
        }
    }
    float4* w = wide + 8 * (size_t)r;
    for (int k = 0; k < 6; ++k) w[k] = o[k];
    w[6] = make_float4(__int_as_float(X.ref[0]), __int_as_float(X.ref[1]), __int_as_float(gref[0]), __int_as_float(gref[1]));
    w[7] = make_float4(__int_as_float(gref[2]), __int_as_float(gref[3]), 0.0f, 0.0f);
    if (!ok) atomicOr(bad, 1u);
}

// ---- multi-GPU: pack owned pixels / scatter a rank's pixels ------------------------------
__global__ void k_pack(const float* fb, const uint32_t* pix, uint32_t P, float* out) {
    uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const float* s = fb + 3 * (size_t)pix[p];
    out[3 * (size_t)p] = s[0];
    out[3 * (size_t)p + 1] = s[1];
    out[3 * (size_t)p + 2] = s[2];
}
__global__ void k_unpack(float* fb, const uint32_t* pix, uint32_t P, const float* in) {
    uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    float* d = fb + 3 * (size_t)pix[p];
    d[0] = in[3 * (size_t)p];
    d[1] = in[3 * (size_t)p + 1];
    d[2] = in[3 * (size_t)p + 2];
}

// ============================================================================
//  host side
// ============================================================================


#define HIPCHK(expr)                                                                                     \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess) return fail(KHP_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define KHPCHK(expr)                \
    do {                            \
        khp_status s_ = (expr);     \
        if (s_ != KHP_OK) return s_; \
    } while (0)

struct TimedLaunch {
    int kind;  // 0 extend, 1 shade, 2 shadow (any hit), 3 other, 4 shadow finish
    int bounce;
    hipEvent_t a, b;
};

// One set of in-flight paths: its own SoA wavefront state, queue counters,
// shadow queues, traversal spill columns and stream pair (A: generate /
// extend / shade / accumulate; B: the shadow stage).
struct PathSet {
    size_t cap = 0;
    DevMem qbuf[2][7], ht, hslot, TFq[2], CKq[2], CKb, shb[2], visb[2], shqb, cnt, spill, spill_sh;
    DevMem heavyb;
    DevMem permb, hkeyb, hclsb;   // shade_order 1
    DevMem lvb;                   // light-path variant: subpath vertices of a chunk's sample slots
    DevMem plane, pspill;         // k_path: per-lane path state columns, traversal-stack spill columns
    DevMem pixo, pixcnt;          // path_order 2: this batch's heavy-first pixel list, its two cursors
    DevMem rs_cols, rs_qsrc, rs_hist, rs_keys;   // ray sorting: regrouped ray columns, state slots, cell counts, cells
    size_t sh_cap = 0;            // shadow-record capacity per parity (cap x connections per path)
    hipStream_t sA = nullptr, sB = nullptr;
};
// Device bytes per path of a PathSet (ensure_wave): 2 x 7 queue columns, hit
// t/slot, TF + CK records, heavy flag, 2 x (occlusion flag + 96-B shadow record: the
// light-path variant's size; next-event records use 64 of it).
constexpr size_t PATH_BYTES = 2 * 7 * 4 + 2 * 4 + 5 * 16 + 1 + 2 * (1 + 6 * 16) + 4 + 1;

#ifndef KHP_MAX_INFLIGHT
#define KHP_MAX_INFLIGHT 3
#endif
struct Snap {
    uint32_t bounce;
};
// One frame slot: the events of the frame last enqueued on its path sets.
struct FrameSlot {
    std::vector<hipEvent_t> ev_pool, sync_pool;  // timing / ordering events, reused per frame
    size_t ev_next = 0, sync_next = 0;
    std::vector<TimedLaunch> launches;
    std::vector<Snap> snaps;
    hipEvent_t ev_start = nullptr, done_t = nullptr, done = nullptr;
    bool inflight = false;
    uint32_t nf = 1;  // frames fused in this slot's batch
};
// An asynchronous operation waiting to be fused into the next batch.
struct PendingOp {
    enum Kind { RENDER, GATHER, SNAPSHOT } kind;
    khp_render_params p;
    int root;
    uint64_t snap = 0;   // SNAPSHOT: khp_read_rgba8_async ticket
};
// ABI 8: an asynchronous 8-bit texture of the running mean (khp_read_rgba8_async).
// k_rgba8 writes dbuf in stream order behind the frames enqueued before it; the
// D2H copy lands in pinned memory; khp_snapshot_wait / khp_sync copy it to the
// caller's buffer.
struct Snapshot {
    uint64_t id = 0;
    uint8_t* out = nullptr;       // caller's W*H*4 bytes
    size_t bytes = 0;
    DevMem dbuf;
    uint8_t* pinned = nullptr;
    hipEvent_t done = nullptr;
    bool enqueued = false;
    bool touched = false;   // an asynchronous operation on dbuf / pinned was queued (snapshot_now)
};
static hipEvent_t slot_event(std::vector<hipEvent_t>& pool, size_t& next, bool no_timing) {
    if (next == pool.size()) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, no_timing ? hipEventDisableTiming : hipEventDefault) != hipSuccess) return nullptr;
        pool.push_back(e);
    }
    return pool[next++];
}

struct khp_ctx {
    int device = 0;
    uint32_t flags = 0;
    hipStream_t stream = nullptr;
    std::vector<hipEvent_t> sync_pool;  // ordering events (no timing)
    int n_cu = 256;
    HostScene hs;
    bool scene_set = false, built = false;
    DevMem prims, aux, trinrm, trifrm, nodes, mats, lights, trislot;
    DevMem wide, wide_bad;   // two-level node records (KHP_WIDE), the build's union check flag
    DevMem topn;             // the top three levels' records for the LDS-staged instances (k_top_nodes)
    DevMem triuv, coneh, texd, texels, mtex;   // ABI 6 textures
    DevScene S{};
    khp_ctx_params prm{};
    khp_bdpt_params bd{};   // light-path variant (ABI 7), off by default
    size_t auto_chunk = 0;         // chunk_paths() when prm.chunk_paths == 0
    // wavefront: one path set per frame slot (ps[0] also serves the batch query API)
    PathSet ps[KHP_MAX_INFLIGHT];
    FrameSlot fs[KHP_MAX_INFLIGHT];
    uint64_t frame_no = 0;
    hipEvent_t fb_evt = nullptr;   // the last framebuffer operation enqueued (accumulate or gather)
    bool report_open = false;      // c->st accumulates harvested frames
    hipEvent_t gather_evt = nullptr;  // end of the last framebuffer gather (becomes fb_evt)
    hipEvent_t snap_evt = nullptr;    // end of the last snapshot's conversion (becomes fb_evt)
    std::vector<PendingOp> pend;      // asynchronous renders (+ gathers, snapshots) not yet enqueued (frame fusion)
    std::vector<Snapshot*> snaps;     // ABI 8 snapshots not yet delivered, oldest first
    std::vector<Snapshot*> snap_free; // buffers of delivered snapshots, for reuse
    uint64_t snap_next = 1;
    hipEvent_t report_ref = nullptr;  // time origin of the open report
    std::vector<std::pair<float, float>> ext_iv;  // the report's k_extend intervals (ms from report_ref)
    // framebuffer + pixel list
    DeviceObjects obj;        // device-flattened objects (device path)
    bool scene_on_host = false;
    DeviceTree tree;          // device-built BVH (preorder nodes, ids), kept for khp_read_bvh
    bool tree_on_device = false;
    uint32_t n_dnodes = 0, n_slots = 0;
    DevMem fb, pix, stage, stage_pix, snap;   // snap: per-bounce Counters snapshots (stats renders)
    DevMem pixheavy;                          // path_order 2: per image pixel, its last camera ray was long
    int cur_bounce = -1;
    std::vector<float> dump;   // prm.dump_bounce: SoA o.xyz, d.xyz of one bounce's extension queue
    std::vector<float> dump_sh;  // prm.dump_bounce: that bounce's shadow rays, o.xyz d.xyz t_max each
    uint32_t fbW = 0, fbH = 0;
    std::vector<uint32_t> pix_host;
    uint32_t pix_key[5] = {0, 0, 0, 0, 0};
    // timing
    std::vector<hipEvent_t> ev_pool;
    size_t ev_next = 0;
    std::vector<TimedLaunch> launches;
    int grid_ext = 0, grid_ext_w = 0, grid_ext_cam = 0, grid_sh = 0, grid_shade = 0;  // k_extend: 64-B, wide, bounce 0
    int grid_fin = 0;    // k_shadow_finish
    int grid_shade_bd = 0;   // k_shade with the light-path variant (512-thread blocks)
    int grid_sh_w = 0;     // k_shadow on the two-level records
    int grid_path = 0, grid_path_w = 0;   // k_path (64-B / two-level records)
    uint32_t bsdf_kinds = 0;              // the BSDF kinds the scene's materials use (bit per khp_bsdf_kind)
    int grid_ext_max = 0;  // the k_extend spill columns are sized for the largest grid
    khp_stats st{};
    // rccl gather: pixel lists cached per (W, H, tile, nranks, rank, root)
    uint32_t gather_key[6] = {0, 0, 0, 0, 0, 0};
    std::vector<uint64_t> gather_counts; // khp_gather_plan counts: root: per sender; sender: its own
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    // ABI 11: while a comm is active (or after it was aborted) every device wait
    // polls with this bound and ncclCommGetAsyncError instead of blocking
    uint32_t comm_timeout_ms = 120000;
    std::string comm_dead;   // why the comm was aborted ("" while alive or never created)
    std::shared_ptr<void> comm_job;   // the init's arguments (CommInitJob), kept while the comm lives
    // RCCL operations enqueued on the stream, oldest first: `pre` is recorded just
    // before the operation (it can run once pre has completed), `post` just after.
    // The bound of a device wait counts only the time an operation has been
    // runnable without completing: compute alone never times out.
    struct CommOp {
        hipEvent_t pre = nullptr, post = nullptr;
        bool runnable = false;
        std::chrono::steady_clock::time_point since;
    };
    std::deque<CommOp> comm_ops;
    std::vector<hipEvent_t> comm_evt_free;
    // khp_read_rgba8's buffers, kept between calls (no allocation per texture):
    // device 8-bit texture, Yxy, block maxima, log terms; pinned host copies of
    // the log terms and maxima; one event per log-term chunk
    DevMem tm_out, tm_yxy, tm_bmax, tm_lgv;
    double* tm_hl = nullptr;
    float* tm_hm = nullptr;
    size_t tm_hl_n = 0, tm_hm_n = 0;
    hipEvent_t tm_ev[16] = {};
    // ABI 8 in-process group (khp_comm_init_local): the gather's transport between
    // contexts of one process instead of RCCL; a sender's k-th gather packs into
    // ring slot k % LG_SLOTS, the root's k-th gather copies every sender's slot k.
    // Sender-side slot state: lg_evts[k] = end of the pack, lg_copied[k] = end of
    // the root's copy (recorded by the root on its stream), lg_stamp[k] = seq + 1
    // of the gather packed there (0: never), lg_taken[k] = the root has enqueued
    // that copy, lg_count[k] = pixels packed.
    std::shared_ptr<std::vector<khp_ctx*>> lgroup;
    DevMem lg_slots[64];
    hipEvent_t lg_evts[64] = {}, lg_copied[64] = {};
    uint64_t lg_stamp[64] = {}, lg_count[64] = {};
    bool lg_taken[64] = {};
    uint64_t lg_seq = 0;
    // render-ahead (khp_ctx_params.render_ahead, ABI 13; k_path's Ahead): the work a
    // synchronous path-kernel call did for the next call of its progressive series
    uint64_t gen = 1;   // bumped by every change of the scene, camera or parameters
    struct AheadSet {
        DevMem st, ck, park;         // AheadState; per ring slot: colour column, park list
        bool valid = false;          // the ring's slot `own` holds the set of the call `next`
        uint32_t own = 0, nsets = 0, park_cap = 0;
        khp_render_params next{};
        uint64_t gen = 0;
        size_t npaths = 0;
        uint32_t* hst = nullptr;     // pinned: AheadState::report of the current call
        bool counted = false;        // hst was filled by the current call
    } ra;
    // render-ahead through fusion (the wavefront's synchronous calls): a call that
    // continues its progressive series renders the next render_ahead calls' passes in
    // the same fused batch; their colours stay in ps[0]'s colour column until those
    // calls accumulate them (wave_ahead_hit).  Any other use of ps[0] drops the batch.
    struct WaveAhead {
        bool valid = false;
        khp_render_params next{};    // the call whose pass is the batch's next frame
        uint64_t gen = 0;
        Wave Wv{};                   // the batch's view: colour column, pixel list, frames' first samples
        uint32_t nf = 0, used = 0;   // frames in the batch, frames accumulated so far
    } wa;
    struct {   // the last synchronous single-pass call, first_sample advanced by its spp
        bool valid = false;
        khp_render_params next{};
        uint64_t gen = 0;
    } series;
};
constexpr size_t LG_SLOTS = 64;

static khp_status drain(khp_ctx* c);
static void comm_release(khp_ctx* c);

// ---- bounded device waits (ABI 11) ------------------------------------------------------------
// Without a communicator a wait blocks (hipEventSynchronize / hipStreamSynchronize).
// With one, the context's stream can hold RCCL sends/receives that only finish when
// the peers post theirs, so a lost or mismatched peer would hang the caller: the
// wait then polls, checks ncclCommGetAsyncError, and after comm_timeout_ms aborts
// the communicator (ncclCommAbort releases its kernels) and fails naming this rank
// and its peers.  KIRK has no multi-device path; its only failure mode is the loud
// exit of CPU_PathTracer.cpp:236-240, which this mirrors as a status.
#ifdef KHP_COMM_TRACE   // diagnostic builds only (tools/build_variant.sh): RCCL steps to stderr
#define COMM_TRACE(...) do { fprintf(stderr, "[khp comm %.3f] ", std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count()); fprintf(stderr, __VA_ARGS__); fprintf(stderr, "\n"); fflush(stderr); } while (0)
#else
#define COMM_TRACE(...) do { } while (0)
#endif
static std::string comm_who(const khp_ctx* c) {
    return "rank " + std::to_string(c->rank) + " of " + std::to_string(c->nranks);
}
static khp_status comm_abort(khp_ctx* c, const std::string& why) {
    if (c->comm) {
        COMM_TRACE("ncclCommAbort begin");
        (void)ncclCommAbort(c->comm);
        COMM_TRACE("ncclCommAbort end");
        c->comm = nullptr;
    }
    c->comm_dead = why;
    return fail(KHP_EDEVICE, why);
}
static bool bounded_waits(const khp_ctx* c) { return c->comm != nullptr || !c->comm_dead.empty(); }

// Brackets of an RCCL operation on the context stream (CommOp).
static hipError_t comm_evt(khp_ctx* c, hipEvent_t* e) {
    if (!c->comm_evt_free.empty()) {
        *e = c->comm_evt_free.back();
        c->comm_evt_free.pop_back();
        return hipSuccess;
    }
    return hipEventCreateWithFlags(e, hipEventDisableTiming);
}
static hipError_t comm_op_begin(khp_ctx* c) {
    khp_ctx::CommOp op;
    hipError_t e = comm_evt(c, &op.pre);
    if (e != hipSuccess) return e;
    e = hipEventRecord(op.pre, c->stream);
    if (e != hipSuccess) {
        c->comm_evt_free.push_back(op.pre);
        return e;
    }
    c->comm_ops.push_back(op);
    return hipSuccess;
}
static hipError_t comm_op_end(khp_ctx* c) {
    khp_ctx::CommOp& op = c->comm_ops.back();
    hipError_t e = comm_evt(c, &op.post);
    if (e != hipSuccess) return e;
    return hipEventRecord(op.post, c->stream);
}
// The oldest RCCL operation that has not completed, after retiring the
// completed ones (nullptr: none in flight).  An operation whose `post` was never
// recorded (its enqueue failed) is retired once its `pre` has completed.
static khp_ctx::CommOp* comm_op_pending(khp_ctx* c) {
    while (!c->comm_ops.empty()) {
        khp_ctx::CommOp& op = c->comm_ops.front();
        const hipError_t q = hipEventQuery(op.post ? op.post : op.pre);
        if (q == hipErrorNotReady) return &op;
        for (hipEvent_t e : {op.pre, op.post})
            if (e) c->comm_evt_free.push_back(e);
        c->comm_ops.pop_front();
    }
    return nullptr;
}

template <typename Query>
static khp_status poll_wait(khp_ctx* c, Query query, const char* what) {
    for (int spins = 0;; ++spins) {
        const hipError_t q = query();
        if (q == hipSuccess) return KHP_OK;
        if (q != hipErrorNotReady) return fail(KHP_EDEVICE, std::string(what) + ": " + hipGetErrorString(q));
        if (c->comm) {
            ncclResult_t ae = ncclSuccess;
            const ncclResult_t r = ncclCommGetAsyncError(c->comm, &ae);
            if (r != ncclSuccess || (ae != ncclSuccess && ae != ncclInProgress))
                return comm_abort(c, comm_who(c) + ": RCCL error while waiting for " + what + ": " +
                                         ncclGetErrorString(r != ncclSuccess ? r : ae) + "; communicator aborted");
        }
        // the bound counts only the time the oldest pending RCCL operation has been
        // runnable (its preceding work done) without completing: a wait on
        // compute alone is never cut short, however long it takes
        khp_ctx::CommOp* op = comm_op_pending(c);
        double ms = 0.0;
        if (op) {
            const auto now = std::chrono::steady_clock::now();
            if (!op->runnable && hipEventQuery(op->pre) == hipSuccess) {
                op->runnable = true;
                op->since = now;
            }
            if (op->runnable) ms = std::chrono::duration<double, std::milli>(now - op->since).count();
        }
        if (ms > c->comm_timeout_ms) {
            if (!c->comm)
                return fail(KHP_EDEVICE, comm_who(c) + ": " + what + " still running " +
                                             std::to_string(c->comm_timeout_ms) + " ms after the communicator abort (" +
                                             c->comm_dead + ")");
            std::string peers;
            for (int r = 0; r < c->nranks; ++r)
                if (r != c->rank) peers += (peers.empty() ? "" : ",") + std::to_string(r);
            return comm_abort(c, comm_who(c) + ": " + what + " not complete after " +
                                     std::to_string(c->comm_timeout_ms) + " ms; a framebuffer gather with peer(s) " +
                                     peers + " is not progressing (a peer lost or its gathers mismatched); "
                                     "communicator aborted");
        }
        if (spins < 256) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}
static khp_status wait_event(khp_ctx* c, hipEvent_t e, const char* what) {
    if (!bounded_waits(c)) {
        HIPCHK(hipEventSynchronize(e));
        return KHP_OK;
    }
    return poll_wait(c, [e] { return hipEventQuery(e); }, what);
}
static khp_status wait_stream(khp_ctx* c, hipStream_t s, const char* what) {
    if (!bounded_waits(c)) {
        HIPCHK(hipStreamSynchronize(s));
        return KHP_OK;
    }
    return poll_wait(c, [s] { return hipStreamQuery(s); }, what);
}

static hipEvent_t next_event(khp_ctx* c) {
    if (c->ev_next == c->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->ev_pool.push_back(e);
    }
    return c->ev_pool[c->ev_next++];
}

// Ordering event k of this render (created once, reused across renders).
static hipEvent_t sync_event(khp_ctx* c, size_t k) {
    while (c->sync_pool.size() <= k) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        c->sync_pool.push_back(e);
    }
    return c->sync_pool[k];
}

extern "C" int khp_abi_version(void) { return KHP_ABI_VERSION; }
extern "C" const char* khp_last_error(void) { return last_error(); }

extern "C" void khp_ctx_params_defaults(khp_ctx_params* out) {
    if (!out) return;
    *out = khp_ctx_params{};
    out->fuse_frames = 32;      // 8 -> 470, 16 -> 485, 32 -> 497 Msamples/s
    out->frames_in_flight = 1;  // with fusion one batch at a time is fastest
    out->chunk_paths = 0;       // min(2^28, fits in half the free HBM)
    out->heavy_iters = 0xFFFFFFFFu;   // longest-first split off (round 6: +0.4% driver, +0.6% 8-spp sync calls, ranks
                                      // unchanged, profiles/r06zzb_heavy_split_off.txt); 160 before
    out->dump_bounce = -1;
    out->trace_kernels = 0;
    out->shade_order = 0;       // hit sorting measured, off
    out->serial_stages = 0;
    out->path_order = 1;       // pixel-major fused chunks, +5-7%
    out->wide_from = KHP_WIDE_FROM;  // two-level records from bounce 2
    out->path_kernel = 0;       // automatic: k_path for synchronous renders
    out->ray_sort_from = 0;     // automatic: bounces 2.. of large trees, +1.8% on the metric row
    out->lds_nodes = 0;         // the top records in LDS, measured
    out->render_ahead = 3;      // a synchronous path-kernel call fills its drain with the next 3 calls' paths,
                                // a wavefront call that continues its series renders the next 3 passes in its batch
}

extern "C" khp_status khp_get_params(khp_ctx* c, khp_ctx_params* out) {
    if (!c || !out) return fail(KHP_EINVAL, "null argument");
    *out = c->prm;
    return KHP_OK;
}

extern "C" khp_status khp_set_params(khp_ctx* c, const khp_ctx_params* prm) {
    if (!c || !prm) return fail(KHP_EINVAL, "null argument");
    if (prm->fuse_frames < 1 || prm->fuse_frames > KHP_MAX_FUSE) return fail(KHP_EINVAL, "fuse_frames must be 1..32");
    if (prm->frames_in_flight < 1 || prm->frames_in_flight > KHP_MAX_INFLIGHT)
        return fail(KHP_EINVAL, "frames_in_flight must be 1..3");
    if (prm->chunk_paths != 0 && prm->chunk_paths < 4096) return fail(KHP_EINVAL, "chunk_paths must be 0 or >= 4096");
    if (prm->chunk_paths > ((uint64_t)1 << 31)) return fail(KHP_EINVAL, "chunk_paths must be <= 2^31");
    if (prm->trace_kernels > 2) return fail(KHP_EINVAL, "trace_kernels must be 0, 1 or 2");
    if (prm->shade_order > 1) return fail(KHP_EINVAL, "shade_order must be 0 or 1");
    if (prm->serial_stages > 1) return fail(KHP_EINVAL, "serial_stages must be 0 or 1");
    if (prm->path_order > 2) return fail(KHP_EINVAL, "path_order must be 0, 1 or 2");
    if (prm->path_kernel > 2) return fail(KHP_EINVAL, "path_kernel must be 0, 1 or 2");
    if (prm->lds_nodes != 0 && prm->lds_nodes != TOP_NODES) return fail(KHP_EINVAL, "lds_nodes must be 0 or 7");
    if (prm->render_ahead > RA_MAX_SETS - 1) return fail(KHP_EINVAL, "render_ahead must be 0..3");
    if (prm->path_from > 64) return fail(KHP_EINVAL, "path_from must be 0..64");
    HIPCHK(hipSetDevice(c->device));
    khp_status dr = drain(c);  // frames in flight finish with the parameters they started with
    if (dr != KHP_OK) return dr;
    c->prm = *prm;
    c->auto_chunk = 0;
    ++c->gen;
    return KHP_OK;
}

extern "C" void khp_bdpt_params_defaults(khp_bdpt_params* out) {
    if (!out) return;
    *out = khp_bdpt_params{};
    out->enabled = 0;
    out->light_paths = 256;
    out->vertices = 4;
    out->bias = 1e-4f;         // the GLSL's 1e-4 bounce bias (pt_shade.compute:269)
    out->bounce_bias = 1e-4f;
    out->min_pdf = 1e-4f;      // SimpleShader's pdf <= 1E-4 cut (SimpleShader.h)
    out->image_plane = 1;      // both GLSL passes: shadeBDPTImagePlane (target as written) and the hit connections
}

extern "C" khp_status khp_get_bdpt(khp_ctx* c, khp_bdpt_params* out) {
    if (!c || !out) return fail(KHP_EINVAL, "null argument");
    *out = c->bd;
    return KHP_OK;
}

extern "C" khp_status khp_set_bdpt(khp_ctx* c, const khp_bdpt_params* p) {
    if (!c || !p) return fail(KHP_EINVAL, "null argument");
    if (p->enabled && (p->light_paths < 1 || p->light_paths > 65536))
        return fail(KHP_EINVAL, "light_paths must be 1..65536");
    if (p->enabled && (p->vertices < 1 || p->vertices > 16)) return fail(KHP_EINVAL, "vertices must be 1..16");
    if (p->image_plane > 2) return fail(KHP_EINVAL, "image_plane must be 0, 1 or 2");
    HIPCHK(hipSetDevice(c->device));
    khp_status dr = drain(c);  // frames in flight finish with the estimator they started with
    if (dr != KHP_OK) return dr;
    c->bd = *p;
    ++c->gen;
    return KHP_OK;
}

extern "C" khp_status khp_set_camera(khp_ctx* c, const khp_camera* cam) {
    if (!c || !cam) return fail(KHP_EINVAL, "null argument");
    HIPCHK(hipSetDevice(c->device));
    khp_status dr = drain(c);  // frames in flight finish with the camera they started with
    if (dr != KHP_OK) return dr;
    c->hs.cam = *cam;
    c->S.cam = *cam;
    ++c->gen;
    return KHP_OK;
}

extern "C" khp_status khp_create(khp_ctx** out, int device, uint32_t flags) {
    if (!out) return fail(KHP_EINVAL, "out is null");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(KHP_EDEVICE, "no HIP device available");
    if (device < 0 || device >= n) return fail(KHP_EINVAL, "device ordinal out of range");
    HIPCHK(hipSetDevice(device));
    khp_ctx* c = new khp_ctx();
    c->device = device;
    c->flags = flags;
    khp_ctx_params_defaults(&c->prm);
    khp_bdpt_params_defaults(&c->bd);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->n_cu = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return fail(KHP_EDEVICE, "hipStreamCreate failed");
    }
    *out = c;
    return KHP_OK;
}

extern "C" void khp_destroy(khp_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)drain(c);
    if (c->stream) (void)wait_stream(c, c->stream, "the context stream at khp_destroy");
    if (c->gather_evt) (void)hipEventDestroy(c->gather_evt);
    if (c->snap_evt) (void)hipEventDestroy(c->snap_evt);
    if (c->report_ref) (void)hipEventDestroy(c->report_ref);
    if (c->lgroup)
        for (auto& m : *c->lgroup)
            if (m == c) m = nullptr;
    for (auto* ev : {c->lg_evts, c->lg_copied})
        for (size_t k = 0; k < 64; ++k)
            if (ev[k]) (void)hipEventDestroy(ev[k]);
    for (auto& w : c->ps) {
        for (hipStream_t s : {w.sA, w.sB}) {
            if (!s) continue;
            (void)wait_stream(c, s, "a frame stream at khp_destroy");
            (void)hipStreamDestroy(s);
        }
    }
    for (auto& f : c->fs) {
        for (auto e : f.ev_pool) (void)hipEventDestroy(e);
        for (auto e : f.sync_pool) (void)hipEventDestroy(e);
    }
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    for (auto e : c->sync_pool) (void)hipEventDestroy(e);
    if (c->tm_hl) (void)hipHostFree(c->tm_hl);
    if (c->tm_hm) (void)hipHostFree(c->tm_hm);
    if (c->ra.hst) (void)hipHostFree(c->ra.hst);
    for (hipEvent_t e : c->tm_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto* v : {&c->snaps, &c->snap_free})
        for (Snapshot* sn : *v) {
            if (sn->pinned) (void)hipHostFree(sn->pinned);
            if (sn->done) (void)hipEventDestroy(sn->done);
            delete sn;
        }
    comm_release(c);   // after every wait above: those still poll while the comm is alive
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

static bool host_path(const khp_ctx* c) { return (c->flags & KHP_CTX_HOST_BUILD) != 0; }

// khp_set_scene_device reads the per-object arrays from device memory but the
// tables (materials, lights, cone_models, textures and their texels,
// material_textures) on the host: cone_models is inverted on the host
// (scene_models), the textures are validated and packed there.  A device
// pointer in one of those fields is refused instead of dereferenced.
static bool is_device_ptr(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // plain (unregistered) host memory
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

static const char* device_table_field(const khp_scene* s) {
    if (is_device_ptr(s->materials)) return "materials";
    if (is_device_ptr(s->lights)) return "lights";
    if (is_device_ptr(s->cone_models)) return "cone_models";
    if (is_device_ptr(s->textures)) return "textures";
    if (is_device_ptr(s->material_textures)) return "material_textures";
    for (uint32_t i = 0; s->textures && i < s->n_textures; ++i)
        if (is_device_ptr(s->textures[i].data)) return "textures[].data";
    return nullptr;
}

static khp_status set_scene_impl(khp_ctx* c, const khp_scene* s, bool device_ptrs) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c) return fail(KHP_EINVAL, "ctx is null");
    auto t0 = std::chrono::steady_clock::now();
    const bool host = host_path(c);
    if (host && device_ptrs) return fail(KHP_EUNSUPPORTED, "device scene arrays need the device build path");
    if (device_ptrs && s) {
        HIPCHK(hipSetDevice(c->device));
        if (const char* f = device_table_field(s))
            return fail(KHP_EINVAL, std::string("khp_set_scene_device: ") + f + " must be host memory");
    }
    c->scene_set = false;
    c->built = false;
    ++c->gen;
    std::string err = flatten_scene(s, c->hs, host);
    if (!err.empty()) return fail(KHP_EINVAL, err);
    c->st.flatten_kernel_ms = 0.0;
    if (host) {
        c->obj.release();
    } else {
        HIPCHK(hipSetDevice(c->device));
        err = device_flatten(s, device_ptrs, s->n_materials, c->hs.textured, c->hs.models, c->obj, c->stream,
                             &c->st.flatten_kernel_ms);
        if (!err.empty()) {
            if (err.rfind("EINVAL:", 0) == 0) return fail(KHP_EINVAL, err.substr(7));
            return fail(KHP_EDEVICE, err);
        }
    }
    c->scene_set = true;
    c->scene_on_host = host;
    c->st.flatten_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->st.build_ms = c->st.flatten_ms;
    return KHP_OK;
}

extern "C" khp_status khp_set_scene(khp_ctx* c, const khp_scene* s) { return set_scene_impl(c, s, false); }

extern "C" khp_status khp_set_scene_device(khp_ctx* c, const khp_scene* s) { return set_scene_impl(c, s, true); }

extern "C" khp_status khp_gen_hairball_device(khp_ctx* c, uint32_t n, uint32_t verts, const float center[3],
                                              float ball_r, float root_r, uint32_t seed, float* d_base_r0,
                                              float* d_apex_r1) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || !center || (n && (!d_base_r0 || !d_apex_r1)) || verts < 2 || verts > 64)
        return fail(KHP_EINVAL, "bad hairball arguments");
    HIPCHK(hipSetDevice(c->device));
    std::string err = device_gen_hairball(n, verts, center, ball_r, root_r, seed, d_base_r0, d_apex_r1, c->stream);
    if (!err.empty()) return fail(KHP_EDEVICE, err);
    return KHP_OK;
}

extern "C" khp_status khp_gen_hairball_tris_device(khp_ctx* c, uint32_t n, uint32_t verts, const float center[3],
                                                   float ball_r, float root_r, uint32_t seed, uint32_t res,
                                                   float* d_v, float* d_n, float* d_frame) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || !center || (n && (!d_v || !d_n || !d_frame)) || verts < 2 || verts > 64 || res == 0)
        return fail(KHP_EINVAL, "bad hairball arguments");
    HIPCHK(hipSetDevice(c->device));
    std::string err = device_gen_hairball_tris(n, verts, center, ball_r, root_r, seed, res, d_v, d_n, d_frame, c->stream);
    if (!err.empty()) return fail(KHP_EDEVICE, err);
    return KHP_OK;
}

extern "C" khp_status khp_device_alloc(khp_ctx* c, size_t bytes, void** out) {
    if (!c || !out) return fail(KHP_EINVAL, "null argument");
    HIPCHK(hipSetDevice(c->device));
    *out = nullptr;
    hipError_t e = hipMalloc(out, bytes ? bytes : 16);
    if (e != hipSuccess) return fail(KHP_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return KHP_OK;
}

extern "C" khp_status khp_device_free(khp_ctx* c, void* p) {
    if (!c) return fail(KHP_EINVAL, "ctx is null");
    if (p) HIPCHK(hipFree(p));
    return KHP_OK;
}

extern "C" khp_status khp_device_copy(khp_ctx* c, void* dst, const void* src, size_t bytes, int to_device) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || (bytes && (!dst || !src))) return fail(KHP_EINVAL, "null argument");
    HIPCHK(hipSetDevice(c->device));
    if (bytes)
        HIPCHK(hipMemcpyAsync(dst, src, bytes, to_device ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, c->stream));
    KHPCHK(wait_stream(c, c->stream, "a device copy"));
    return KHP_OK;
}

template <typename T>
static hipError_t upload(DevMem& m, const T* data, size_t count, hipStream_t s) {
    hipError_t e = m.ensure(count * sizeof(T));
    if (e != hipSuccess) return e;
    if (count) return hipMemcpyAsync(m.p, data, count * sizeof(T), hipMemcpyHostToDevice, s);
    return hipSuccess;
}

extern "C" khp_status khp_build_accel(khp_ctx* c) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c) return fail(KHP_EINVAL, "ctx is null");
    if (!c->scene_set) return fail(KHP_ENOTREADY, "khp_set_scene first");
    HIPCHK(hipSetDevice(c->device));
    auto t0 = std::chrono::steady_clock::now();
    const bool host_build = c->scene_on_host;  // the path khp_set_scene flattened on
    HostScene& hs = c->hs;
    c->built = false;
    c->st.bvh_kernel_ms = 0.0;
    c->st.bvh_on_device = host_build ? 0u : 1u;
    double lay_kernel_ms = 0.0;
    int32_t root_ref = 0, root_cnt = 0;
    float root_box[6];
    uint32_t n_dnodes = 0, n_slots = 0;
    std::chrono::steady_clock::time_point tb, t1;
    if (host_build) {
        c->tree_on_device = false;
        unsigned nt = std::thread::hardware_concurrency();
        build_bvh(hs, (int)std::max(1u, std::min(nt, 32u)));
        tb = std::chrono::steady_clock::now();
        make_device_layout(hs);
        t1 = std::chrono::steady_clock::now();
        n_dnodes = (uint32_t)hs.dnodes.size();
        n_slots = hs.n_slots;
        if (n_slots >= MAX_SLOTS)
            return fail(KHP_EUNSUPPORTED, "more than 2^24 primitive slots do not fit the packed leaf reference");
        HIPCHK(upload(c->prims, hs.slot_rec.data(), hs.slot_rec.size(), c->stream));
        HIPCHK(upload(c->aux, hs.slot_aux.data(), hs.slot_aux.size(), c->stream));
        HIPCHK(upload(c->nodes, hs.dnodes.data(), hs.dnodes.size(), c->stream));
        root_ref = hs.root_ref;
        root_cnt = hs.root_cnt;
        memcpy(root_box, hs.root_box, sizeof(root_box));
        c->st.n_nodes = hs.nodes.size();
        c->tree.release();
    } else {
        // the tree stays in HBM; hs.nodes / hs.ids are filled only on khp_read_bvh
        hs.nodes.clear();
        hs.ids.clear();
        hs.dnodes.clear();
        hs.slot_rec.clear();
        hs.slot_aux.clear();
        std::string err = device_build_bvh(hs, c->obj, c->stream, c->tree, &c->st.bvh_kernel_ms);
        if (!err.empty()) return fail(KHP_EDEVICE, err);
        c->tree_on_device = true;
        tb = std::chrono::steady_clock::now();
        DeviceLayout lay;
        err = device_layout(c->obj, c->tree, c->stream, c->nodes, c->prims, c->aux, lay, &lay_kernel_ms);
        if (!err.empty()) return fail(KHP_EDEVICE, err);
        t1 = std::chrono::steady_clock::now();
        n_dnodes = lay.n_dnodes;
        n_slots = lay.n_slots;
        if (n_slots >= MAX_SLOTS)
            return fail(KHP_EUNSUPPORTED, "more than 2^24 primitive slots do not fit the packed leaf reference");
        root_ref = lay.root_ref;
        root_cnt = lay.root_cnt;
        memcpy(root_box, lay.root_box, sizeof(root_box));
        c->st.n_nodes = c->tree.n_nodes;
        c->st.layout_kernel_ms = lay_kernel_ms;
    }
    c->st.bvh_ms = std::chrono::duration<double, std::milli>(tb - t0).count();
    c->st.layout_ms = std::chrono::duration<double, std::milli>(t1 - tb).count();
    c->st.build_ms = c->st.flatten_ms + c->st.bvh_ms + c->st.layout_ms;
    if (hs.depth + 1 > (uint32_t)STACK_MAX)
        return fail(KHP_EUNSUPPORTED, "BVH deeper than the traversal stack (" + std::to_string(hs.depth) + ")");
    if (host_build) {
        HIPCHK(upload(c->trinrm, hs.tri_nrm.data(), hs.tri_nrm.size(), c->stream));
        HIPCHK(upload(c->trifrm, hs.tri_frame.data(), hs.tri_frame.size(), c->stream));
    }
    HIPCHK(upload(c->mats, hs.mats.data(), hs.mats.size(), c->stream));
    HIPCHK(upload(c->lights, hs.lights.data(), hs.lights.size(), c->stream));
    if (hs.textured) {
        if (host_build) {
            HIPCHK(upload(c->triuv, hs.tri_uv.data(), hs.tri_uv.size(), c->stream));
            HIPCHK(upload(c->coneh, hs.cone_h.data(), hs.cone_h.size(), c->stream));
        }
        HIPCHK(upload(c->texd, hs.tex.data(), hs.tex.size(), c->stream));
        HIPCHK(upload(c->texels, hs.texels.data(), hs.texels.size(), c->stream));
        HIPCHK(upload(c->mtex, hs.mtex.data(), hs.mtex.size(), c->stream));
    }
    // Two-level node records for k_extend (traverse.h iterw), when every node's
    // box is the union of its children's (always, for KIRK's build).
    bool wide_ok = false;
    if (KHP_WIDE && n_dnodes > 0) {
        HIPCHK(c->wide.ensure((size_t)n_dnodes * 8 * sizeof(float4)));
        HIPCHK(c->wide_bad.ensure(sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(c->wide_bad.p, 0, sizeof(uint32_t), c->stream));
        hipLaunchKernelGGL(k_wide_records, dim3((n_dnodes + 255) / 256), dim3(256), 0, c->stream,
                           c->nodes.as<DevNode>(), n_dnodes, c->wide.as<float4>(), c->wide_bad.as<uint32_t>());
        HIPCHK(hipGetLastError());
        uint32_t bad = 1;
        HIPCHK(hipMemcpyAsync(&bad, c->wide_bad.p, sizeof(bad), hipMemcpyDeviceToHost, c->stream));
        KHPCHK(wait_stream(c, c->stream, "the scene build"));
        wide_ok = bad == 0;
    }
    if (!wide_ok) c->wide.release();
    if (n_dnodes > 0) {   // the top-of-tree records for khp_ctx_params.lds_nodes
        HIPCHK(c->topn.ensure(TOP_NODES * sizeof(DevNode)));
        hipLaunchKernelGGL(k_top_nodes, dim3(1), dim3(64), 0, c->stream, c->nodes.as<DevNode>(), root_ref,
                           c->topn.as<DevNode>());
        HIPCHK(hipGetLastError());
    }
    HIPCHK(c->trislot.ensure(4 * (size_t)std::max(hs.n_tris, 1u)));
    if (hs.n_tris > 0 && n_slots > 0)
        hipLaunchKernelGGL(k_tri_slots, dim3((n_slots + 255) / 256), dim3(256), 0, c->stream, c->prims.as<float4>(),
                           c->aux.as<Aux>(), n_slots, hs.n_tris, c->trislot.as<uint32_t>());
    HIPCHK(hipGetLastError());
    KHPCHK(wait_stream(c, c->stream, "the scene build"));
    c->st.upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    DevScene& S = c->S;
    S.tri_slot = c->trislot.as<uint32_t>();
    S.prims = c->prims.as<float4>();
    S.aux = c->aux.as<Aux>();
    S.tri_nrm = host_build ? c->trinrm.as<float>() : c->obj.tri_nrm.as<float>();
    S.tri_frame = host_build ? c->trifrm.as<float>() : c->obj.tri_frame.as<float>();
    S.nodes = c->nodes.as<DevNode>();
    S.wide = wide_ok ? c->wide.as<float4>() : nullptr;
    S.top = n_dnodes > 0 ? c->topn.as<float4>() : nullptr;
    S.top_root = n_dnodes > 0 && ((uint32_t)root_ref & LEAF_BIT) == 0u ? (int32_t)TOP_REF : root_ref;
    S.mats = c->mats.as<khp_material>();
    S.lights = c->lights.as<DevLight>();
    S.n_lights = (int32_t)hs.lights.size();
    S.root_ref = root_ref;
    S.root_cnt = root_cnt;
    memcpy(S.root_box, root_box, sizeof(S.root_box));
    c->n_dnodes = n_dnodes;
    c->n_slots = n_slots;
    S.env = hs.env;
    S.cam = hs.cam;
    S.textured = hs.textured ? 1 : 0;
    S.n_tris = hs.n_tris;
    S.env_map = hs.env_map;
    S.tri_uv = !hs.textured ? nullptr : host_build ? c->triuv.as<float>() : c->obj.tri_uv.as<float>();
    S.cone_h = !hs.textured ? nullptr : host_build ? c->coneh.as<float>() : c->obj.cone_h.as<float>();
    S.tex = hs.textured ? c->texd.as<DevTexture>() : nullptr;
    S.texels = hs.textured ? c->texels.as<uint8_t>() : nullptr;
    S.mtex = hs.textured ? c->mtex.as<DevMatTex>() : nullptr;
    c->st.n_objects = hs.n_obj;
    c->st.n_leaves = (c->st.n_nodes + 1) / 2;
    c->st.bvh_depth = hs.depth;
    c->st.max_leaf_size = hs.max_leaf;
    c->st.device_bytes = c->prims.bytes + c->aux.bytes + c->trinrm.bytes + c->trifrm.bytes + c->nodes.bytes + c->wide.bytes + c->mats.bytes +
                         c->lights.bytes;
    // persistent grid sizes
    int nb = 0;
    if (c->flags & KHP_CTX_STATS)
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_extend<true>, TRAV_BLOCK, EXT_LDS_BYTES));
    else
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_extend<false>, TRAV_BLOCK, EXT_LDS_BYTES));
    c->grid_ext = std::max(1, nb) * c->n_cu;
    nb = 0;
    if (c->flags & KHP_CTX_STATS)
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_extend<true, false, true>, TRAV_BLOCK, EXT_LDS_BYTES));
    else
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_extend<false, false, true>, TRAV_BLOCK, EXT_LDS_BYTES));
    c->grid_ext_w = std::max(1, nb) * c->n_cu;
    nb = 0;
    if (c->flags & KHP_CTX_STATS)
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_extend<true, true>, TRAV_BLOCK, CAM_LDS_BYTES));
    else
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_extend<false, true>, TRAV_BLOCK, CAM_LDS_BYTES));
    c->grid_ext_cam = std::max(1, nb) * c->n_cu;
    c->grid_ext_max = std::max(c->grid_ext, std::max(c->grid_ext_w, c->grid_ext_cam));
    nb = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_shadow<false>, TRAV_BLOCK, LDS_BYTES));
    c->grid_sh = std::max(1, nb) * c->n_cu;
    nb = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_shadow<false, true>, TRAV_BLOCK, LDS_BYTES));
    c->grid_sh_w = std::min(c->grid_sh, std::max(1, nb) * c->n_cu);  // the spill columns are sized by grid_sh
    c->bsdf_kinds = 0;   // the kinds the materials use: fur scenes run kernels with the others compiled out
    for (const khp_material& m : hs.mats)
        c->bsdf_kinds |= (m.bsdf >= 0 && m.bsdf < KHP_BSDF_COUNT) ? (1u << m.bsdf) : KINDS_ALL;
    nb = 0;
    if (S.textured) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_shade<true, false>), shade_block<true, false>(), 0));
    else if ((c->bsdf_kinds & ~KINDS_FUR) == 0u)
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_shade<false, false, KINDS_FUR>), shade_block<false, false>(), 0));
    else HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_shade<false, false>), shade_block<false, false>(), 0));
    c->grid_shade = std::max(1, nb) * c->n_cu;
    nb = 0;
    if (S.textured) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_shade<true, true>), shade_block<true, true>(), 0));
    else HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_shade<false, true>), shade_block<false, true>(), 0));
    c->grid_shade_bd = std::max(1, nb) * c->n_cu;
    // k_shadow_finish streams shadow records in 256-thread blocks: its own occupancy grid
    // (k_shade's 512-thread grid gave it 0.4x the threads: 0.333 vs 0.314 ms per frame)
    nb = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_shadow_finish<false>), 256, 0));
    c->grid_fin = std::max(1, nb) * c->n_cu;
    nb = 0;
    if (S.textured) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_path<true, false, KINDS_ALL, true>), TRAV_BLOCK, PATH_LDS));
    else HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_path<false, false, KINDS_ALL, true>), TRAV_BLOCK, PATH_LDS));
    c->grid_path = std::max(1, nb) * c->n_cu;
    nb = 0;
    if (S.textured) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_path<true, true, KINDS_ALL, true>), TRAV_BLOCK, PATH_LDS));
    else HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (k_path<false, true, KINDS_ALL, true>), TRAV_BLOCK, PATH_LDS));
    c->grid_path_w = std::min(c->grid_path, std::max(1, nb) * c->n_cu);   // the columns are sized by grid_path
    c->built = true;
    ++c->gen;
    return KHP_OK;
}

static khp_status ensure_wave(khp_ctx* c, PathSet& w, size_t cap, size_t sh_per_path = 1) {
    if (cap <= w.cap && cap * sh_per_path <= w.sh_cap) return KHP_OK;
    cap = std::max(cap, w.cap);
    const size_t shc = std::max(cap * sh_per_path, w.sh_cap);
    for (int q = 0; q < 2; ++q)
        for (int k = 0; k < 7; ++k) HIPCHK(w.qbuf[q][k].ensure(cap * 4));
    HIPCHK(w.ht.ensure(cap * 4));
    HIPCHK(w.hslot.ensure(cap * 4));
    for (int q = 0; q < 2; ++q) {
        HIPCHK(w.TFq[q].ensure(cap * sizeof(float4)));
        HIPCHK(w.CKq[q].ensure(cap * sizeof(float4)));
    }
    HIPCHK(w.CKb.ensure(cap * sizeof(float4)));
    HIPCHK(w.heavyb.ensure(cap));
    HIPCHK(w.permb.ensure(cap * 4));
    HIPCHK(w.hkeyb.ensure(cap));
    HIPCHK(w.hclsb.ensure(32 * 4));
    for (int q = 0; q < 2; ++q) {
        HIPCHK(w.visb[q].ensure(shc));
        HIPCHK(w.shb[q].ensure(shc * 6 * sizeof(float4)));
    }
    w.sh_cap = shc;
    HIPCHK(w.shqb.ensure(2 * sizeof(ShadowQ)));
    HIPCHK(w.cnt.ensure(sizeof(Counters)));
    // traversal-stack spill columns: one per resident lane, STACK_MAX entries deep
    // separate spill columns: k_extend and k_shadow may run at the same time
    HIPCHK(w.spill.ensure((size_t)c->grid_ext_max * TRAV_BLOCK * STACK_MAX * sizeof(int4)));
    HIPCHK(w.spill_sh.ensure((size_t)c->grid_sh * TRAV_BLOCK * STACK_MAX * sizeof(int4)));
    if (!w.sA) {
        HIPCHK(hipStreamCreateWithFlags(&w.sA, hipStreamNonBlocking));
        HIPCHK(hipStreamCreateWithFlags(&w.sB, hipStreamNonBlocking));
    }
    w.cap = cap;
    return KHP_OK;
}

// Device pointers of the wavefront state (sized by ensure_wave).
static Wave wave_view(const khp_ctx* c, PathSet& w) {
    Wave Wv{};
    for (int q = 0; q < 2; ++q) {
        for (int k = 0; k < 3; ++k) {
            Wv.qo[q][k] = w.qbuf[q][k].as<float>();
            Wv.qd[q][k] = w.qbuf[q][3 + k].as<float>();
        }
        Wv.qpid[q] = w.qbuf[q][6].as<uint32_t>();
    }
    Wv.ht = w.ht.as<float>();
    Wv.hslot = w.hslot.as<int32_t>();
    for (int q = 0; q < 2; ++q) {
        Wv.TFq[q] = w.TFq[q].as<float4>();
        Wv.CKq[q] = w.CKq[q].as<float4>();
    }
    Wv.CK = w.CKb.as<float4>();
    Wv.vis = w.visb[0].as<uint8_t>();
    Wv.sh = w.shb[0].as<float4>();
    Wv.shs = 6;
    Wv.shq = w.shqb.as<ShadowQ>();
    Wv.cnt = w.cnt.as<Counters>();
    Wv.heavy = w.heavyb.as<uint8_t>();
    Wv.cap = (uint32_t)w.cap;
    Wv.heavy_T = c->prm.heavy_iters;
    Wv.perm = c->prm.shade_order ? w.permb.as<uint32_t>() : nullptr;
    Wv.hkey = w.hkeyb.as<uint8_t>();
    Wv.hcls = w.hclsb.as<uint32_t>();
    return Wv;
}

static khp_status prepare_pixels(khp_ctx* c, const khp_render_params* p) {
    uint32_t T = p->tile_size ? p->tile_size : 64;
    uint32_t nranks = p->tile_nranks > 1 ? p->tile_nranks : 1;
    uint32_t rank = nranks > 1 ? p->tile_rank : 0;
    uint32_t key[5] = {p->width, p->height, T, rank, nranks};
    if (memcmp(key, c->pix_key, sizeof(key)) == 0 && c->pix.p) return KHP_OK;
    owned_pixels(p->width, p->height, T, rank, nranks, c->pix_host);
    HIPCHK(upload(c->pix, c->pix_host.data(), c->pix_host.size(), c->stream));
    memcpy(c->pix_key, key, sizeof(key));
    return KHP_OK;
}

// Paths per wavefront chunk.  A chunk's path state is PATH_BYTES (~350 B) per
// path, ~95 GB at 2^28.  By default the smaller of 2^28 and the largest power of
// two whose path sets (one per batch in flight) fit in half the free HBM; with
// the 5/4 rule of chunk_most the driver's 20 fused 8-spp passes at the metric
// row (332M paths) are then ONE chunk: each launch's tail is paid once per 20
// frames, +1.8% against two chunks of 166M under the round-5 cap of 2^27
// (profiles/r06zi_one_chunk_ab.txt).
// Decided once per context (and again after khp_set_params), before the path
// sets themselves take memory, so the chunking stays the same frame to frame.
static size_t chunk_paths(khp_ctx* c) {
    if (c->prm.chunk_paths) return (size_t)c->prm.chunk_paths;
    if (c->auto_chunk) return c->auto_chunk;
    size_t free_b = 0, total_b = 0;
    size_t cap = (size_t)1 << 28;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b) {
        const size_t fit = free_b / 2 / (PATH_BYTES * (size_t)std::max<uint32_t>(1, c->prm.frames_in_flight));
        while (cap > ((size_t)1 << 16) && cap > fit) cap >>= 1;
    }
    c->auto_chunk = cap;
    return cap;
}

// The most paths one fused chunk may hold: the cap, or with automatic chunking
// 5/4 of it (enqueue_frames cuts a batch into one chunk fewer when the chunks
// then stay within this; flush() groups gathered frames by the same limit).
static size_t chunk_most(khp_ctx* c) {
    const size_t cap = chunk_paths(c);
    return cap + (c->prm.chunk_paths == 0 ? cap / 4 : 0);
}

static khp_status check_params(khp_ctx* c, const khp_render_params* p) {
    if (!c || !p) return fail(KHP_EINVAL, "null argument");
    if (!c->built) return fail(KHP_ENOTREADY, "khp_build_accel first");
    if (p->width == 0 || p->height == 0 || p->depth == 0) return fail(KHP_EINVAL, "width/height/depth must be > 0");
    if ((uint64_t)p->width * p->height >= (1ull << 31)) return fail(KHP_EINVAL, "image too large");
    uint32_t T = p->tile_size ? p->tile_size : 64;
    if (T % 8 != 0) return fail(KHP_EINVAL, "tile_size must be a multiple of 8");
    if (p->tile_nranks > 1 && p->tile_rank >= p->tile_nranks) return fail(KHP_EINVAL, "tile_rank >= tile_nranks");
    return KHP_OK;
}

static void timed(khp_ctx* c, FrameSlot& f, int kind, bool begin, hipStream_t st) {
    hipEvent_t e = slot_event(f.ev_pool, f.ev_next, false);
    if (!e) return;
    (void)hipEventRecord(e, st);
    if (begin) f.launches.push_back(TimedLaunch{kind, c->cur_bounce, e, nullptr});
    else f.launches.back().b = e;
}

// Zero the per-report fields of c->st (timings, counters, per-bounce tables).
static void report_begin(khp_ctx* c) {
    c->st.render_ms = 0.0;
    c->st.extend_ms = c->st.shade_ms = c->st.shadow_ms = c->st.other_ms = 0.0;
    c->st.extend_launches = 0;
    c->st.shadow_launches = 0;
    c->st.shadow_finish_ms = 0.0;
    c->st.extend_rays = c->st.shadow_rays = c->st.node_visits = c->st.prim_tests = 0;
    c->st.shadow_node_visits = c->st.shadow_prim_tests = c->st.stack_spills = 0;
    c->st.extend_pruned_pops = c->st.shadow_pruned_pops = 0;
    for (int q = 0; q < 4; ++q) c->st.step_cycles[q] = 0;
    for (int k = 0; k < KHP_MAX_BOUNCE_STATS; ++k) {
        c->st.bounce_extend_ms[k] = c->st.bounce_shadow_ms[k] = 0.0;
        c->st.bounce_rays[k] = c->st.bounce_nodes[k] = c->st.bounce_prims[k] = 0;
        c->st.bounce_shadow_rays[k] = c->st.bounce_shadow_nodes[k] = c->st.bounce_shadow_prims[k] = 0;
        c->st.bounce_wave_iters[k] = c->st.bounce_lanes_busy[k] = 0;
        c->st.bounce_shadow_wave_iters[k] = c->st.bounce_shadow_lanes_busy[k] = 0;
    }
    c->st.frames = 0;
    c->st.extend_busy_ms = 0.0;
    c->st.ahead_finished = c->st.ahead_resumed = 0;
    c->ext_iv.clear();
    if (!c->report_ref) (void)hipEventCreate(&c->report_ref);
    (void)hipEventRecord(c->report_ref, c->stream);
    c->report_open = true;
}

// Union of the report's k_extend intervals (ms).
static double union_ms(std::vector<std::pair<float, float>>& iv) {
    std::sort(iv.begin(), iv.end());
    double tot = 0.0, lo = 0.0, hi = -1.0;
    for (auto& x : iv) {
        if (x.first > hi) {
            if (hi > lo) tot += hi - lo;
            lo = x.first;
            hi = x.second;
        } else if (x.second > hi) {
            hi = x.second;
        }
    }
    if (hi > lo) tot += hi - lo;
    return tot;
}

// Wait for one in-flight frame and add its timings and counters to the open report.
static khp_status harvest(khp_ctx* c, int slot) {
    FrameSlot& f = c->fs[slot];
    if (!f.inflight) return KHP_OK;
    f.inflight = false;
    KHPCHK(wait_event(c, f.done, "a batch of frames"));
    if (!c->report_open) report_begin(c);
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, f.ev_start, f.done_t) == hipSuccess) c->st.render_ms += ms;
    c->st.frames += f.nf;
    c->st.subframes = 1;
    for (auto& l : f.launches) {
        float t = 0.0f;
        if (l.b && hipEventElapsedTime(&t, l.a, l.b) == hipSuccess) {
            if (l.kind == 0) {
                c->st.extend_ms += t;
                c->st.extend_launches++;
                float t0 = 0.0f, t1 = 0.0f;
                if (hipEventElapsedTime(&t0, c->report_ref, l.a) == hipSuccess &&
                    hipEventElapsedTime(&t1, c->report_ref, l.b) == hipSuccess)
                    c->ext_iv.push_back({t0, t1});
            }
            else if (l.kind == 1) c->st.shade_ms += t;
            else if (l.kind == 2) {
                c->st.shadow_ms += t;
                c->st.shadow_launches++;
            } else if (l.kind == 4) {
                c->st.shadow_ms += t;
                c->st.shadow_finish_ms += t;
            } else {
                c->st.other_ms += t;
            }
            if (l.bounce >= 0 && l.bounce < KHP_MAX_BOUNCE_STATS) {
                if (l.kind == 0) c->st.bounce_extend_ms[l.bounce] += t;
                if (l.kind == 2 || l.kind == 4) c->st.bounce_shadow_ms[l.bounce] += t;
            }
        }
    }
    {
        Counters hc;
        HIPCHK(hipMemcpy(&hc, c->ps[slot].cnt.p, sizeof(hc), hipMemcpyDeviceToHost));
        c->st.extend_rays += hc.ext_rays;
        c->st.shadow_rays += hc.sh_rays;
        c->st.node_visits += hc.node_visits;
        c->st.prim_tests += hc.prim_tests;
        c->st.shadow_node_visits += hc.sh_node_visits;
        c->st.shadow_prim_tests += hc.sh_prim_tests;
        c->st.stack_spills += hc.spills;
        c->st.extend_pruned_pops += hc.pruned;
        c->st.shadow_pruned_pops += hc.sh_pruned;
        for (int q = 0; q < 4; ++q) c->st.step_cycles[q] += hc.step_cycles[q];
    }
    c->st.extend_busy_ms = union_ms(c->ext_iv);
    if (!f.snaps.empty()) {
        std::vector<Counters> sn(f.snaps.size());
        HIPCHK(hipMemcpy(sn.data(), c->snap.p, sn.size() * sizeof(Counters), hipMemcpyDeviceToHost));
        Counters pv{};   // counters after the previous snapshot
        for (size_t i = 0; i < sn.size(); ++i) {
            const uint32_t b = f.snaps[i].bounce;
            if (b < KHP_MAX_BOUNCE_STATS) {
                c->st.bounce_rays[b] += sn[i].ext_rays - pv.ext_rays;
                c->st.bounce_nodes[b] += sn[i].node_visits - pv.node_visits;
                c->st.bounce_prims[b] += sn[i].prim_tests - pv.prim_tests;
                c->st.bounce_shadow_rays[b] += sn[i].sh_rays - pv.sh_rays;
                c->st.bounce_shadow_nodes[b] += sn[i].sh_node_visits - pv.sh_node_visits;
                c->st.bounce_shadow_prims[b] += sn[i].sh_prim_tests - pv.sh_prim_tests;
                c->st.bounce_wave_iters[b] += sn[i].iters - pv.iters;
                c->st.bounce_lanes_busy[b] += sn[i].lanes_busy - pv.lanes_busy;
                c->st.bounce_shadow_wave_iters[b] += sn[i].sh_iters - pv.sh_iters;
                c->st.bounce_shadow_lanes_busy[b] += sn[i].sh_lanes_busy - pv.sh_lanes_busy;
            }
            pv = sn[i];
        }
        f.snaps.clear();
    }
    return KHP_OK;
}

// Wait for every in-flight frame (their stats go to the open report) and for
// the context stream.  Every entry point that reads or replaces device state
// other than through an asynchronous render calls this first.
static khp_status flush(khp_ctx* c);
static khp_status drain(khp_ctx* c) {
    khp_status fr = flush(c);
    if (fr != KHP_OK) return fr;
    for (int s = 0; s < KHP_MAX_INFLIGHT; ++s) {
        khp_status r = harvest(c, s);
        if (r != KHP_OK) return r;
    }
    if (c->stream) KHPCHK(wait_stream(c, c->stream, "the context stream"));
    return KHP_OK;
}

static khp_status deliver_snapshots(khp_ctx* c, uint64_t upto, bool wait);

extern "C" khp_status khp_sync(khp_ctx* c) {
    if (!c) return fail(KHP_EINVAL, "null context");
    HIPCHK(hipSetDevice(c->device));
    if (!c->report_open) report_begin(c);
    khp_status s = drain(c);
    c->report_open = false;
    if (s != KHP_OK) return s;
    return deliver_snapshots(c, UINT64_MAX, true);
}

// Enqueue one frame, or a fused batch of asynchronous frames (ops: their
// render operations, which differ only in first_sample, and the framebuffer
// gathers between them, in call order; p = the first render's parameters).
static khp_status gather_now(khp_ctx* c, const khp_render_params* p, int root);
static khp_status snapshot_now(khp_ctx* c, uint64_t id);
// A non-render operation of a fused batch, in call order.
static khp_status op_now(khp_ctx* c, const PendingOp& o) {
    return o.kind == PendingOp::SNAPSHOT ? snapshot_now(c, o.snap) : gather_now(c, &o.p, o.root);
}
// Render-ahead (k_path's Ahead): the call p of npaths paths in one chunk.  When
// the previous such call rendered ahead for exactly this call (same scene,
// camera, parameters, pixels, spp, depth, seed; first_sample = its own +
// spp), its ahead set becomes this call's own set -- its finished colours,
// claim cursors and parked paths -- otherwise both sets start empty.  The
// other parity is cleared for this call's ahead set.  Enqueued on s before the
// launch; ahead_commit records the set once the launch is enqueued.
static bool ahead_key_equal(const khp_render_params& a, const khp_render_params& b) {
    return a.width == b.width && a.height == b.height && a.spp == b.spp && a.depth == b.depth && a.seed == b.seed &&
           a.first_sample == b.first_sample && a.tile_size == b.tile_size && a.tile_rank == b.tile_rank &&
           a.tile_nranks == b.tile_nranks;
}
static khp_status ahead_prepare(khp_ctx* c, const khp_render_params* p, size_t npaths, hipStream_t s, Ahead& A,
                                float4** ck_own) {
    khp_ctx::AheadSet& ra = c->ra;
    const uint32_t nsets = std::min<uint32_t>(c->prm.render_ahead, RA_MAX_SETS - 1) + 1;
    const bool match = ra.valid && ra.gen == c->gen && ra.npaths == npaths && ra.nsets == nsets &&
                       ahead_key_equal(ra.next, *p);
    ra.valid = false;
    // a lane parks at most one path per launch, and a set is parked by the nsets - 1
    // launches before the one it belongs to
    const size_t lanes = (size_t)c->grid_path * TRAV_BLOCK;
    const size_t cap = (nsets - 1) * lanes;
    HIPCHK(ra.st.ensure(sizeof(AheadState)));
    HIPCHK(ra.ck.ensure(nsets * npaths * sizeof(float4)));
    HIPCHK(ra.park.ensure(nsets * cap * PARK_F4 * sizeof(float4)));
    uint32_t clear;
    if (match) {   // the previous call's next set is this call's own set; its own slot takes the farthest set
        clear = 1u << ra.own;
        ra.own = (ra.own + 1) % nsets;
    } else {
        clear = (1u << RA_MAX_SETS) - 1u;
        ra.own = 0;
    }
    ra.nsets = nsets;
    ra.park_cap = (uint32_t)cap;
    AheadState* st = ra.st.as<AheadState>();
    A = Ahead{};
    A.on = 1u;
    A.npaths = (uint32_t)npaths;
    A.spp = p->spp;
    A.own = ra.own;
    A.nsets = nsets;
    A.park_cap = (uint32_t)cap;
    A.st = st;
    A.ck = ra.ck.as<float4>();
    A.park = ra.park.as<float4>();
    hipLaunchKernelGGL(k_ahead_prep, dim3(1), dim3(256), 0, s, st, clear, ra.own);
    if (!ra.hst) HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&ra.hst), 2 * sizeof(uint32_t), hipHostMallocDefault));
    HIPCHK(hipMemcpyAsync(ra.hst, st->report, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    ra.counted = true;
    *ck_own = ra.ck.as<float4>() + (size_t)ra.own * npaths;
    return KHP_OK;
}
static void ahead_commit(khp_ctx* c, const khp_render_params* p, size_t npaths) {
    khp_ctx::AheadSet& ra = c->ra;
    ra.valid = true;
    ra.next = *p;
    ra.next.first_sample = p->first_sample + p->spp;
    ra.gen = c->gen;
    ra.npaths = npaths;
}

// Render-ahead through fusion: the synchronous call p is the next frame of the
// batch an earlier call of its series rendered (same scene, camera, parameters,
// pixels, spp, depth, seed; first_sample = that call's + j spp).  Its paths are
// done; the call only folds their colours into the running mean (k_accumulate
// of frame j, the kernel a fused batch runs per frame) -- the framebuffer is the
// one the call renders alone, bit for bit.
static khp_status wave_ahead_hit(khp_ctx* c, const khp_render_params* p, float* out_rgb) {
    khp_ctx::WaveAhead& wa = c->wa;
    const uint32_t P = wa.Wv.P;
    hipEvent_t e0 = next_event(c), e1 = next_event(c);
    (void)hipEventRecord(e0, c->stream);
    if (c->fb_evt) HIPCHK(hipStreamWaitEvent(c->stream, c->fb_evt, 0));
    hipLaunchKernelGGL(k_accumulate, dim3((P + 255) / 256), dim3(256), 0, c->stream, wa.Wv, c->fb.as<float>(), wa.used);
    HIPCHK(hipGetLastError());
    (void)hipEventRecord(e1, c->stream);
    ++wa.used;
    wa.next.first_sample = p->first_sample + p->spp;
    if (wa.used >= wa.nf) wa.valid = false;
    if (out_rgb && !(p->flags & KHP_RENDER_NO_READBACK)) {
        hipMemcpyKind kind = (p->flags & KHP_RENDER_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        HIPCHK(hipMemcpyAsync(out_rgb, c->fb.p, (size_t)p->width * p->height * 3 * sizeof(float), kind, c->stream));
    }
    KHPCHK(wait_stream(c, c->stream, "a synchronous frame"));
    float ms = 0.0f;
    if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess) c->st.render_ms = ms;
    c->st.other_ms = ms;
    c->ev_next = 0;
    c->st.frames = 1;
    c->st.ahead_finished = (uint64_t)P * p->spp;
    c->report_open = false;
    c->series.valid = true;
    c->series.next = *p;
    c->series.next.first_sample = p->first_sample + p->spp;
    c->series.gen = c->gen;
    return KHP_OK;
}

static khp_status enqueue_frames(khp_ctx* c, const khp_render_params* p, float* out_rgb,
                                 const std::vector<PendingOp>* ops) {
    khp_status s;
    const bool stats = (c->flags & KHP_CTX_STATS) != 0 || (p->flags & KHP_RENDER_STATS) != 0;
    const bool async = (p->flags & KHP_RENDER_ASYNC) != 0;
    // fused frames: their first samples, in call order
    std::vector<uint32_t> fs0;
    if (ops) {
        for (const PendingOp& o : *ops)
            if (o.kind == PendingOp::RENDER) fs0.push_back(o.p.first_sample);
    } else {
        fs0.push_back(p->first_sample);
    }
    uint32_t nf = (uint32_t)fs0.size();
    const size_t npix = (size_t)p->width * p->height;
    uint32_t T = p->tile_size ? p->tile_size : 64;
    uint32_t nranks = p->tile_nranks > 1 ? p->tile_nranks : 1;
    uint32_t pkey[5] = {p->width, p->height, T, nranks > 1 ? p->tile_rank : 0u, nranks};
    const bool geometry_change = c->fbW != p->width || c->fbH != p->height || !c->fb.p ||
                                 memcmp(pkey, c->pix_key, sizeof(pkey)) != 0 || !c->pix.p;
    if (!async || geometry_change) {  // a synchronous render (or new buffers) first completes the in-flight frames
        s = drain(c);
        if (s != KHP_OK) return s;
        // An asynchronous frame on new buffers keeps accumulating into the
        // report opened since the last khp_sync; only a synchronous render
        // starts a fresh one.
        if (!async) c->report_open = false;
    }
    if (!async) report_begin(c);
    else if (!c->report_open) report_begin(c);
    // render-ahead through fusion (c->wa): a synchronous single pass that an earlier
    // call already rendered only accumulates; every other render drops the batch
    const bool sync1 = !async && !ops && nf == 1;
    const bool continues = sync1 && c->series.valid && c->series.gen == c->gen && ahead_key_equal(c->series.next, *p);
    c->series.valid = false;
    if (sync1 && !stats && c->wa.valid && c->wa.gen == c->gen && ahead_key_equal(c->wa.next, *p) && c->fb.p &&
        c->fbW == p->width && c->fbH == p->height)
        return wave_ahead_hit(c, p, out_rgb);
    c->wa.valid = false;
    if (c->fbW != p->width || c->fbH != p->height || !c->fb.p) {
        HIPCHK(c->fb.ensure(npix * 3 * sizeof(float)));
        HIPCHK(hipMemsetAsync(c->fb.p, 0, npix * 3 * sizeof(float), c->stream));
        HIPCHK(c->pixheavy.ensure(npix));
        HIPCHK(hipMemsetAsync(c->pixheavy.p, 0, npix, c->stream));
        c->fbW = p->width;
        c->fbH = p->height;
    }
    s = prepare_pixels(c, p);
    if (s != KHP_OK) return s;
    if (geometry_change) KHPCHK(wait_stream(c, c->stream, "the framebuffer setup"));
    const uint32_t P_all = (uint32_t)c->pix_host.size();
    // Batches in flight: an asynchronous render takes the next frame slot (its
    // own path set and streams) and returns once enqueued; up to
    // prm.frames_in_flight batches then run at the same time, each persistent
    // launch taking 1/F of the resident grid.  The framebuffer is written in
    // render order: each accumulate waits for the previous framebuffer
    // operation (accumulate or gather).
    const int F = (int)std::max<uint32_t>(1, std::min<uint32_t>(c->prm.frames_in_flight, KHP_MAX_INFLIGHT));
    const int slot = async ? (int)(c->frame_no % (uint64_t)F) : 0;
    c->frame_no += async ? 1 : 0;
    s = harvest(c, slot);  // the slot's previous batch (async series)
    if (s != KHP_OK) return s;
    FrameSlot& f = c->fs[slot];
    f.ev_next = 0;
    f.sync_next = 0;
    f.launches.clear();
    f.snaps.clear();
    const int G = async ? F : 1;
    const int grid_ext = std::max(1, c->grid_ext / G), grid_sh = std::max(1, c->grid_sh / G);
    const int grid_sh_w = std::max(1, c->grid_sh_w / G);
    const int grid_ext_w = std::max(1, c->grid_ext_w / G), grid_ext_cam = std::max(1, c->grid_ext_cam / G);
    // Chunks: the owned pixels x samples (x fused frames) are cut into chunks
    // of at most chunk_paths() paths, pixel-major; a fused chunk carries all
    // samples of all frames of its pixels.
    // light-path variant: up to `vertices` connection records per path and bounce,
    // so a chunk carries 1/vertices of the paths (the same shadow-record memory)
    const bool bdm = c->bd.enabled != 0 && c->S.n_lights > 0;
    const uint32_t sh_per_path = bdm ? c->bd.vertices : 1u;
    const size_t cap_paths = std::max<size_t>(4096 / sh_per_path, chunk_paths(c) / sh_per_path);
    const int dump_b = (!async && !ops) ? c->prm.dump_bounce : -1;
    // the path kernel (khp_ctx_params.path_kernel): automatic for synchronous renders of at
    // most PATH_AUTO_MAX paths.  At the metric row a synchronous call of s spp takes
    // 8.0 / 12.5 / 16.7 / 20.8 / 29.4 / 37.6 ms through it for s = 1 / 2 / 3 / 4 / 6 / 8
    // against 14.0 / 17.9 / 21.4 / 24.7 / 31.2 / 37.2 through the wavefront
    // (profiles/r04aa_sync_spp.json): the wavefront's better steady rate wins from ~7.5 spp
    constexpr size_t PATH_AUTO_MAX = (size_t)14 << 20;
    const bool path_ok = !stats && !bdm && c->prm.shade_order == 0 && dump_b < 0;
    // render-ahead through fusion: a synchronous wavefront call that continues its series
    // (the previous synchronous call was its pass with first_sample - spp) renders itself and
    // the next render_ahead calls' passes as one fused batch of one chunk, accumulates its own
    // frame and leaves the others' colours for those calls (8-spp calls at the metric row:
    // a batch of 3 / 4 passes costs 28.6 / 27.5 ms per pass against 36.8 alone,
    // profiles/r06t_fuse_probe.jsonl)
    uint32_t wa_frames = 1;
    if (continues && c->prm.render_ahead != 0 && !stats && !bdm && dump_b < 0 && P_all > 0) {
        const size_t one = (size_t)P_all * p->spp;
        const bool wavefront = !(path_ok && (c->prm.path_kernel == 2 ||
                                             (c->prm.path_kernel == 0 && one <= PATH_AUTO_MAX)));
        const uint32_t F = 1u + std::min<uint32_t>(c->prm.render_ahead, RA_MAX_SETS - 1);
        if (wavefront && one * F <= cap_paths && F <= KHP_MAX_FUSE) wa_frames = F;
    }
    for (uint32_t q = 1; q < wa_frames; ++q) fs0.push_back(p->first_sample + q * p->spp);
    nf = (uint32_t)fs0.size();
    f.nf = nf;
    uint32_t P_chunk, S_chunk;
    if (nf > 1) {
        P_chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(std::max<uint32_t>(1, P_all),
                                                                 cap_paths / ((size_t)p->spp * nf)));
        // equal chunks (in whole 64-pixel blocks where that stays under the cap): 20 fused
        // 8-spp 1080p frames are 3 chunks of 691k pixels instead of 839k + 839k + 395k, so
        // no chunk's launches run a short, tail-dominated wavefront
        uint32_t n_ch = (P_all + P_chunk - 1) / std::max<uint32_t>(1, P_chunk);
        // automatic chunk size: one chunk fewer when the chunks then stay within 5/4
        // of the cap (20 fused 8-spp 1080p frames: 2 chunks of 166M paths instead of
        // 3 of 111M, +1.2% measured; 32 frames stay 4 chunks of 133M)
        if (n_ch > 1 && c->prm.chunk_paths == 0) {
            const uint64_t lo_px = (P_all + (n_ch - 1) - 1) / (n_ch - 1);
            if (lo_px * p->spp * nf <= chunk_most(c) / sh_per_path) {
                --n_ch;
                P_chunk = (uint32_t)lo_px;
            }
        }
        if (n_ch > 1) {
            const uint32_t even = (P_all + n_ch - 1) / n_ch, blk = (even + 63u) & ~63u;
            P_chunk = blk <= P_chunk ? blk : even;
        }
        S_chunk = p->spp;
    } else {
        P_chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(P_all, cap_paths));
        S_chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(p->spp, cap_paths / P_chunk));
    }
    if (ops && (P_chunk < P_all || S_chunk < p->spp)) {
        for (const PendingOp& o : *ops)  // flush() groups gathered frames so that each group is one chunk
            if (o.kind != PendingOp::RENDER)
                return fail(KHP_EINVAL, "internal: a fused batch with gathers or snapshots spans more than one chunk");
    }
    if (bdm && nf == 1) {  // the light subpaths of a chunk's sample slots take at most a quarter of the free HBM
        size_t free_b = 0, total_b = 0;
        const size_t per_slot = (size_t)c->bd.light_paths * c->S.n_lights * c->bd.vertices * 48;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && per_slot)
            S_chunk = (uint32_t)std::max<size_t>(1, std::min<size_t>(S_chunk, free_b / 4 / per_slot));
    }
    // a partial batch (flushed by a sync) reserves room for a full one, so the
    // first full batch does not allocate
    // (automatic chunks may reach 5/4 of the cap, see above)
    size_t want = (size_t)P_chunk * S_chunk * nf;
    if (ops && nf > 1) {
        const uint32_t fuse = std::max<uint32_t>(1, std::min<uint32_t>(c->prm.fuse_frames, KHP_MAX_FUSE));
        want = std::max(want, std::min<size_t>(chunk_most(c) / sh_per_path, (size_t)P_all * S_chunk * fuse));
    }
    PathSet& w = c->ps[slot];
    s = ensure_wave(c, w, want, sh_per_path);
    if (s != KHP_OK) return s;
    // light subpaths of a chunk: one per (frame, sample slot, subpath, light); k_light_paths
    // indexes them with 32 bits, and their vertices (48 B each) must fit beside the path sets
    size_t lv_bytes = 0;
    if (bdm) {
        const uint64_t nsub = (uint64_t)nf * S_chunk * c->bd.light_paths * (uint64_t)c->S.n_lights;
        if (nsub >= ((uint64_t)1 << 31))
            return fail(KHP_EINVAL, "light-path variant: frames x samples x light_paths x lights per chunk reaches "
                                    "2^31 subpaths; lower light_paths or the samples per pass");
        lv_bytes = (size_t)nsub * c->bd.vertices * 48;
        if (lv_bytes > w.lvb.bytes) {
            size_t free_b = 0, total_b = 0;
            if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && lv_bytes + (lv_bytes >> 3) > free_b)
                return fail(KHP_ENOMEM, "light-path variant: " + std::to_string(lv_bytes >> 20) +
                                            " MiB of light vertices per chunk exceed the free HBM; lower light_paths, "
                                            "vertices or the samples per pass");
        }
        HIPCHK(w.lvb.ensure(lv_bytes));
    }
    const size_t call_paths = (size_t)P_all * p->spp * nf;
    const bool use_path = path_ok && (c->prm.path_kernel == 2 ||
                                      (c->prm.path_kernel == 0 && !async && call_paths <= PATH_AUTO_MAX));
    const bool path_wide = use_path && c->S.wide != nullptr && c->prm.wide_from == 0;
    // hybrid batches (khp_ctx_params.path_from): a wavefront render hands the paths still
    // alive at bounce path_from to one k_path launch, which carries them through the
    // remaining bounces without a barrier per bounce (not with the light-path variant,
    // hit sorting, instrumented renders or queue dumps)
    const uint32_t hyb_from = (!use_path && path_ok && c->prm.path_from > 0 && c->prm.path_from < p->depth)
                              ? c->prm.path_from : 0u;
    const bool hyb_wide = hyb_from > 0 && c->S.wide != nullptr && hyb_from >= c->prm.wide_from;
    PathLanes PL{};
    SpillArea sp_path{nullptr, 0};
    if (use_path || hyb_from > 0) {
        const size_t lanes = (size_t)c->grid_path * TRAV_BLOCK;
        HIPCHK(w.plane.ensure(lanes * 8 * sizeof(float4)));
        HIPCHK(w.pspill.ensure(lanes * STACK_MAX * sizeof(int4)));
        for (int k = 0; k < 8; ++k) PL.col[k] = w.plane.as<float4>() + (size_t)k * lanes;
        sp_path = SpillArea{w.pspill.as<int4>(), (uint32_t)lanes};
    }
    const int grid_path = std::max(1, ((path_wide || hyb_wide) ? c->grid_path_w : c->grid_path) / G);
    if (stats) {
        const size_t chunks = (size_t)((P_all + P_chunk - 1) / P_chunk) * ((p->spp + S_chunk - 1) / S_chunk);
        HIPCHK(c->snap.ensure(std::max<size_t>(1, chunks * p->depth) * sizeof(Counters)));
    }
    // Two streams: A runs generate / extend / shade / accumulate, B runs the
    // shadow stage (k_shadow + k_shadow_finish) of bounce b while A already
    // traverses bounce b+1, so each persistent kernel's tail fills with the
    // other's blocks.  Ordering: B(b) after shade(b) on A; shade(b+1) after
    // B(b) (both update the path colour C in bounce order); the shadow queue
    // of bounce b+2 reuses parity b's buffers only after shade(b+1), which
    // already waited for B(b).  Instrumented renders run everything on the
    // context stream so the per-bounce snapshots are exact.
    const bool overlap = !stats && !c->prm.serial_stages;
    hipStream_t sA = overlap ? w.sA : c->stream;
    hipStream_t sB = overlap ? w.sB : c->stream;
    c->cur_bounce = -1;
    f.ev_start = slot_event(f.ev_pool, f.ev_next, false);
    (void)hipEventRecord(f.ev_start, c->stream);
    // Fork from the context stream (framebuffer clears, pixel-list uploads) --
    // not for an asynchronous frame: the context stream also carries the joins
    // of the frames still in flight, and waiting on it would serialise them.
    if (!async || geometry_change) {
        hipEvent_t e_fork = slot_event(f.sync_pool, f.sync_next, true);
        HIPCHK(hipEventRecord(e_fork, c->stream));
        if (sA != c->stream) HIPCHK(hipStreamWaitEvent(sA, e_fork, 0));
        if (sB != c->stream) HIPCHK(hipStreamWaitEvent(sB, e_fork, 0));
    }
    hipEvent_t prev_acc = c->fb_evt;  // the previous framebuffer operation (this batch's accumulate waits for it)
    HIPCHK(hipMemsetAsync(w.cnt.p, 0, sizeof(Counters), sA));
    HIPCHK(hipMemsetAsync(w.shqb.p, 0, 2 * sizeof(ShadowQ), sA));
    if (sB != sA) {
        hipEvent_t z = slot_event(f.sync_pool, f.sync_next, true);
        HIPCHK(hipEventRecord(z, sA));
        HIPCHK(hipStreamWaitEvent(sB, z, 0));
    }
    bool acc_waited = false;
    Wave Wv = wave_view(c, w);
    // render-ahead (khp_ctx_params.render_ahead): synchronous path-kernel calls of one chunk
    const bool ahead = use_path && !async && !ops && nf == 1 && c->prm.render_ahead != 0 && P_all > 0 &&
                       P_chunk >= P_all && S_chunk >= p->spp && call_paths <= (size_t)PID_MASK + 1;
    Ahead AH{};
    if (ahead) KHPCHK(ahead_prepare(c, p, call_paths, sA, AH, &Wv.CK));
    Wv.pix = c->pix.as<uint32_t>();
    Wv.W = p->width;
    Wv.H = p->height;
    Wv.seed = p->seed;
    Wv.depth = p->depth;
    Wv.pix_major = c->prm.path_order != 0 ? 1u : 0u;
    Wv.pixheavy = nullptr;
    if (c->prm.path_order == 2 && !use_path && P_all) {  // heavy-first pixel list (k_pix_order), per path set
        HIPCHK(w.pixo.ensure((size_t)P_all * sizeof(uint32_t)));
        HIPCHK(w.pixcnt.ensure(2 * sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync(w.pixcnt.p, 0, 2 * sizeof(uint32_t), sA));
        hipLaunchKernelGGL(k_pix_order, dim3((P_all + 255) / 256), dim3(256), 0, sA, c->pix.as<uint32_t>(), P_all,
                           c->pixheavy.as<uint8_t>(), w.pixo.as<uint32_t>(), w.pixcnt.as<uint32_t>());
        Wv.pix = w.pixo.as<uint32_t>();
        Wv.pixheavy = c->pixheavy.as<uint8_t>();
    }
    // camera rays in place at bounce 0 (no generate pass): not for the light-path
    // variant (its image-plane connections add to the queued bounce-0 state) nor
    // when bounce 0's queue is dumped
    Wv.cam0 = (!bdm && dump_b != 0) ? 1u : 0u;
    Wv.shs = bdm ? 6u : 4u;   // next-event records are 64 B; the light-path variant's connection records 96
    Wv.bd = BdptDev{bdm ? 1u : 0u, c->bd.light_paths, (uint32_t)c->S.n_lights, c->bd.vertices, c->bd.bias,
                    c->bd.bounce_bias, c->bd.min_pdf, c->bd.image_plane,
                    bdm ? w.lvb.as<float4>() : nullptr};
    // ray sorting from bounce rs_from (0: off); not with hit sorting, the light-path
    // variant or queue dumps, which read the queues in their own order.  Automatic
    // (ray_sort_from 0): from bounce 2 when the node records exceed RS_AUTO_BYTES --
    // a cache-resident tree has no misses to save (config 2: -3.6%, config 1: -17%)
    const uint32_t rs_param = c->prm.ray_sort_from != 0 ? c->prm.ray_sort_from
                              : (uint64_t)c->n_dnodes * sizeof(DevNode) >= RS_AUTO_BYTES ? 2u : 0u;
    const uint32_t rs_from = (c->prm.shade_order == 0 && !bdm && dump_b < 0) ? rs_param : 0u;
    SpillArea sp_ext{w.spill.as<int4>(), (uint32_t)c->grid_ext_max * TRAV_BLOCK};
    SpillArea sp_sh{w.spill_sh.as<int4>(), (uint32_t)c->grid_sh * TRAV_BLOCK};
    for (uint32_t p0 = 0; p0 < P_all; p0 += P_chunk) {
        const uint32_t P = std::min(P_chunk, P_all - p0);
        for (uint32_t s0 = 0; s0 < p->spp; s0 += S_chunk) {
            const uint32_t ns = std::min(S_chunk, p->spp - s0);
            Wv.P = P;
            Wv.p_off = p0;
            Wv.sample0 = fs0[0] + s0;
            Wv.n_samples = ns;
            Wv.n_frames = nf;
            for (uint32_t q = 0; q < nf; ++q) Wv.fsample0[q] = fs0[q] + s0;
            const uint32_t npaths = P * ns * nf;
            if (use_path) {  // every bounce of the chunk's paths in one launch; then the accumulate below
                HIPCHK(hipMemsetAsync(reinterpret_cast<char*>(Wv.cnt) + offsetof(Counters, fetch_ext), 0,
                                      sizeof(Counters::fetch_ext), sA));
                timed(c, f, 3, true, sA);
                launch_path(c->S.textured != 0, path_wide, (c->bsdf_kinds & ~KINDS_FUR) == 0u, grid_path, sA, c->S, Wv,
                            sp_path, PL, AH);
                HIPCHK(hipGetLastError());
                if (ahead) ahead_commit(c, p, call_paths);
                timed(c, f, 3, false, sA);
            }
            timed(c, f, 3, true, sA);
            if (use_path) {
            } else if (Wv.cam0) hipLaunchKernelGGL(k_start, dim3(1), dim3(1), 0, sA, Wv.cnt, npaths);
            else hipLaunchKernelGGL(k_generate, dim3((npaths + 255) / 256), dim3(256), 0, sA, c->S, Wv);
            if (bdm) {  // the light subpaths of this chunk's sample slots (frames x samples)
                const uint32_t nsub = nf * ns * c->bd.light_paths * (uint32_t)c->S.n_lights;
                hipLaunchKernelGGL(k_light_paths, dim3((nsub + 63) / 64), dim3(64), 0, sA, c->S, Wv);
            }
            timed(c, f, 3, false, sA);
            if (bdm && c->bd.image_plane) {
                // shadeBDPTImagePlane before bounce 0, all on stream A: connection groups
                // on the parity-1 shadow buffers, traced, and added to the bounce-0 state
                Wave Wi = Wv;
                Wi.sh = w.shb[1].as<float4>();
                Wi.vis = w.visb[1].as<uint8_t>();
                Wi.shq = w.shqb.as<ShadowQ>() + 1;
                HIPCHK(hipMemsetAsync(Wi.shq, 0, sizeof(ShadowQ), sA));
                hipLaunchKernelGGL(k_img_connect, dim3((npaths + 255) / 256), dim3(256), 0, sA, c->S, Wi);
                timed(c, f, 2, true, sA);
                launch_shadow(stats, false, grid_sh, sA, c->S, Wi, sp_sh);
                timed(c, f, 2, false, sA);
                timed(c, f, 4, true, sA);
                hipLaunchKernelGGL(k_shadow_finish<true>, dim3(c->grid_fin), dim3(256), 0, sA, c->S, Wi, 0);
                timed(c, f, 4, false, sA);
            }
            hipEvent_t done_b = nullptr;  // shadow stage of the previous bounce finished (B)
            bool sorted = false;          // this bounce's queue was regrouped by origin cell (rs_*)
            bool prepped = false;         // this bounce's k_prep was enqueued before the previous fork
            const uint32_t b_stop = use_path ? 0u : hyb_from > 0 ? hyb_from : p->depth;   // wavefront bounces
            for (uint32_t b = 0; b < b_stop; ++b) {
                const int cur = b & 1;
                c->cur_bounce = (int)b;
                Wave Wb = Wv;
                if (sorted) {   // the regrouped ray columns replace this parity's; the state stays put
                    const size_t cp = w.cap;
                    for (int k = 0; k < 3; ++k) {
                        Wb.qo[cur][k] = w.rs_cols.as<float>() + k * cp;
                        Wb.qd[cur][k] = w.rs_cols.as<float>() + (3 + k) * cp;
                    }
                    Wb.qpid[cur] = w.rs_cols.as<uint32_t>() + 6 * cp;
                    Wb.qsrc = w.rs_qsrc.as<uint32_t>();
                }
                Wb.sh = w.shb[cur].as<float4>();
                Wb.vis = w.visb[cur].as<uint8_t>();
                Wb.shq = w.shqb.as<ShadowQ>() + cur;
                if (dump_b == (int)b && p0 == 0 && s0 == 0) {  // extension queue: front part, then back part
                    uint32_t nq[2] = {0, 0};
                    HIPCHK(hipMemcpyAsync(&nq[0], &Wv.cnt->nq[cur], 4, hipMemcpyDeviceToHost, sA));
                    HIPCHK(hipMemcpyAsync(&nq[1], &Wv.cnt->nqb[cur], 4, hipMemcpyDeviceToHost, sA));
                    KHPCHK(wait_stream(c, sA, "the queue dump"));
                    const size_t m = (size_t)nq[0] + nq[1];
                    c->dump.resize(6 * m);
                    for (int q = 0; q < 6; ++q) {
                        const float* col = q < 3 ? Wv.qo[cur][q] : Wv.qd[cur][q - 3];
                        float* dst = c->dump.data() + (size_t)q * m;
                        HIPCHK(hipMemcpy(dst, col, 4 * (size_t)nq[0], hipMemcpyDeviceToHost));
                        HIPCHK(hipMemcpy(dst + nq[0], col + (Wv.cap - nq[1]), 4 * (size_t)nq[1], hipMemcpyDeviceToHost));
                    }
                }
                if (!prepped) hipLaunchKernelGGL(k_prep, dim3(1), dim3(1), 0, sA, Wv.cnt, Wb.shq, cur);
                prepped = false;
#ifdef KHP_LEAF_REUSE
                if (stats) HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_reuse_b), &b, sizeof(b), 0, hipMemcpyHostToDevice, sA));
#endif
                timed(c, f, 0, true, sA);
                const bool cam = b == 0 && Wv.cam0;
                const bool wide = c->S.wide != nullptr && b >= c->prm.wide_from;
                launch_extend(stats, cam, wide, wide ? grid_ext_w : cam ? grid_ext_cam : grid_ext, sA, c->S, Wb, cur,
                              sp_ext, c->prm.lds_nodes != 0);
                timed(c, f, 0, false, sA);
                if (done_b && sB != sA) HIPCHK(hipStreamWaitEvent(sA, done_b, 0));
                timed(c, f, 1, true, sA);
                if (Wb.perm) {  // hit sorting (shade_order 1): part of the shade time
                    HIPCHK(hipMemsetAsync(Wb.hcls, 0, 32 * sizeof(uint32_t), sA));
                    hipLaunchKernelGGL(k_hit_class, dim3(c->grid_shade), dim3(256), 0, sA, c->S, Wb, cur);
                    hipLaunchKernelGGL(k_hit_scatter, dim3(c->grid_shade), dim3(256), 0, sA, Wb, cur);
                }
                if (c->S.textured && bdm)
                    hipLaunchKernelGGL((k_shade<true, true>), dim3(c->grid_shade_bd), dim3(shade_block<true, true>()), 0, sA, c->S, Wb, cur, b);
                else if (c->S.textured)
                    hipLaunchKernelGGL((k_shade<true, false>), dim3(c->grid_shade), dim3(shade_block<true, false>()), 0, sA, c->S, Wb, cur, b);
                else if (bdm)
                    hipLaunchKernelGGL((k_shade<false, true>), dim3(c->grid_shade_bd), dim3(shade_block<false, true>()), 0, sA, c->S, Wb, cur, b);
                else if ((c->bsdf_kinds & ~KINDS_FUR) == 0u)   // fur scenes: the other BSDF kinds compiled out
                    hipLaunchKernelGGL((k_shade<false, false, KINDS_FUR>), dim3(c->grid_shade), dim3(shade_block<false, false>()), 0, sA, c->S, Wb,
                                       cur, b);
                else
                    hipLaunchKernelGGL((k_shade<false, false>), dim3(c->grid_shade), dim3(shade_block<false, false>()), 0, sA, c->S, Wb, cur, b);
                timed(c, f, 1, false, sA);
                // ray sorting: regroup the next bounce's queue by origin cell
                auto sort_next = [&]() -> khp_status {
                    sorted = rs_from > 0 && b + 1 >= rs_from && b + 1 < p->depth;
                    if (sorted) {
                        const size_t cp = w.cap;
                        HIPCHK(w.rs_cols.ensure(7 * cp * sizeof(float)));
                        HIPCHK(w.rs_qsrc.ensure(cp * sizeof(uint32_t)));
                        HIPCHK(w.rs_keys.ensure(cp * sizeof(uint32_t)));
                        HIPCHK(w.rs_hist.ensure(2 * RS_CELLS * sizeof(uint32_t)));
                        uint32_t* hist = w.rs_hist.as<uint32_t>();
                        Wave Wn = Wv;   // the next queue (parity cur ^ 1) as shade wrote it
                        timed(c, f, 3, true, sA);   // under "other": shade_ms stays k_shade's alone
                        HIPCHK(hipMemsetAsync(hist, 0, RS_CELLS * sizeof(uint32_t), sA));
                        const uint32_t rs_per_cu = std::max(1u, std::min(2048u / RS_THREADS, 163840u / (RS_CELLS * 4u)));
                        const dim3 rs_grid((c->n_cu > 0 ? (uint32_t)c->n_cu : 256u) * rs_per_cu);   // resident blocks
                        hipLaunchKernelGGL(k_rsort_count, rs_grid, dim3(RS_THREADS), 0, sA, c->S, Wn, cur ^ 1, hist,
                                           w.rs_keys.as<uint32_t>());
                        hipLaunchKernelGGL(k_rsort_scan, dim3(1), dim3(1024), 0, sA, hist, hist + RS_CELLS);
                        hipLaunchKernelGGL(k_rsort_scatter, rs_grid, dim3(RS_THREADS), 0, sA, Wn, cur ^ 1,
                                           w.rs_keys.as<uint32_t>(), hist + RS_CELLS, w.rs_cols.as<float>(),
                                           w.rs_qsrc.as<uint32_t>());
                        HIPCHK(hipGetLastError());
                        timed(c, f, 3, false, sA);
                    }
                    return KHP_OK;
                };
                KHPCHK(sort_next());   // before the shadow stage forks: alone on the chip it takes ~0.2 ms
                                       // per frame, beside the shadow stage's persistent grid ~2 ms
                if (!stats && sB != sA && b + 1 < p->depth) {
                    // the next bounce's counter reset before the fork, so its k_extend is ready on
                    // stream A when the shadow stage becomes ready on B (the queues it resets are
                    // consumed: this bounce's, and the previous bounce's shadow queue, which
                    // k_shade waited for); +0.4%, profiles/r05ad_early_prep_ab.txt.  Instrumented
                    // renders keep the reset at the bounce's start (per-bounce counter snapshots)
                    hipLaunchKernelGGL(k_prep, dim3(1), dim3(1), 0, sA, Wv.cnt, w.shqb.as<ShadowQ>() + (cur ^ 1),
                                       cur ^ 1);
                    prepped = true;
                }
                if (sB != sA) {
                    hipEvent_t shaded = slot_event(f.sync_pool, f.sync_next, true);
                    HIPCHK(hipEventRecord(shaded, sA));
                    HIPCHK(hipStreamWaitEvent(sB, shaded, 0));
                }
                if (dump_b == (int)b && p0 == 0 && s0 == 0) {  // this bounce's shadow rays: o, d, t_max
                    KHPCHK(wait_stream(c, sA, "the queue dump"));
                    ShadowQ hq;
                    HIPCHK(hipMemcpy(&hq, Wb.shq, sizeof(ShadowQ), hipMemcpyDeviceToHost));
                    const size_t R = Wv.shs;   // float4 per record
                    std::vector<float4> rec(R * ((size_t)hq.nsh + hq.nshb));
                    if (hq.nsh)
                        HIPCHK(hipMemcpy(rec.data(), Wb.sh, R * sizeof(float4) * hq.nsh, hipMemcpyDeviceToHost));
                    if (hq.nshb)
                        HIPCHK(hipMemcpy(rec.data() + R * (size_t)hq.nsh, Wb.sh + R * (Wv.cap - hq.nshb),
                                         R * sizeof(float4) * hq.nshb, hipMemcpyDeviceToHost));
                    c->dump_sh.resize(7 * ((size_t)hq.nsh + hq.nshb));
                    for (size_t k = 0; k < (size_t)hq.nsh + hq.nshb; ++k) {
                        const float4 a = rec[R * k], d = rec[R * k + 1];
                        const float v[7] = {a.x, a.y, a.z, d.x, d.y, d.z, a.w};
                        memcpy(c->dump_sh.data() + 7 * k, v, sizeof(v));
                    }
                }
                timed(c, f, 2, true, sB);
                const bool wide_sh = c->S.wide != nullptr && b >= std::max(c->prm.wide_from, (uint32_t)KHP_WIDE_SH_FROM);
                launch_shadow(stats, wide_sh, wide_sh ? grid_sh_w : grid_sh, sB, c->S, Wb, sp_sh, c->prm.lds_nodes != 0);
                timed(c, f, 2, false, sB);
                timed(c, f, 4, true, sB);   // shadow stage = any-hit traversal + finish
                if (bdm) hipLaunchKernelGGL(k_shadow_finish<true>, dim3(c->grid_fin), dim3(256), 0, sB, c->S, Wb, cur ^ 1);
                else hipLaunchKernelGGL(k_shadow_finish<false>, dim3(c->grid_fin), dim3(256), 0, sB, c->S, Wb, cur ^ 1);
                timed(c, f, 4, false, sB);
                if (sB != sA) {
                    done_b = slot_event(f.sync_pool, f.sync_next, true);
                    HIPCHK(hipEventRecord(done_b, sB));
                }
                if (stats) {
                    HIPCHK(hipMemcpyAsync(c->snap.as<Counters>() + f.snaps.size(), w.cnt.p, sizeof(Counters),
                                          hipMemcpyDeviceToDevice, sA));
                    f.snaps.push_back(Snap{b});
                }
            }
            if (hyb_from > 0) {   // the remaining bounces of the paths in the bounce-hyb_from queue
                const int cur = hyb_from & 1;
                Wave Wq = Wv;
                if (sorted) {   // regrouped: ray columns and state slots as k_extend would take them
                    const size_t cp = w.cap;
                    for (int k = 0; k < 3; ++k) {
                        Wq.qo[cur][k] = w.rs_cols.as<float>() + k * cp;
                        Wq.qd[cur][k] = w.rs_cols.as<float>() + (3 + k) * cp;
                    }
                    Wq.qpid[cur] = w.rs_cols.as<uint32_t>() + 6 * cp;
                    Wq.qsrc = w.rs_qsrc.as<uint32_t>();
                }
                Wq.q_cur = (uint32_t)cur;
                Wq.q_bounce = hyb_from;
                if (done_b && sB != sA) HIPCHK(hipStreamWaitEvent(sA, done_b, 0));   // the deferred colour adds
                if (!prepped) hipLaunchKernelGGL(k_prep, dim3(1), dim3(1), 0, sA, Wv.cnt, w.shqb.as<ShadowQ>() + cur, cur);
                prepped = false;
                c->cur_bounce = (int)hyb_from;
                timed(c, f, 3, true, sA);
                launch_path(c->S.textured != 0, hyb_wide, (c->bsdf_kinds & ~KINDS_FUR) == 0u, grid_path, sA, c->S, Wq,
                            sp_path, PL, Ahead{}, true);
                HIPCHK(hipGetLastError());
                timed(c, f, 3, false, sA);
            }
            c->cur_bounce = -1;
            if (done_b) HIPCHK(hipStreamWaitEvent(sA, done_b, 0));
            if (prev_acc && !acc_waited) {  // framebuffer order: previous frame
                HIPCHK(hipStreamWaitEvent(sA, prev_acc, 0));
                acc_waited = true;
            }
            timed(c, f, 3, true, sA);
            bool only_renders = true;
            if (ops)
                for (const PendingOp& o : *ops) only_renders = only_renders && o.kind == PendingOp::RENDER;
            if (wa_frames > 1) {   // this call's frame; the later frames wait for their calls
                hipLaunchKernelGGL(k_accumulate, dim3((P + 255) / 256), dim3(256), 0, sA, Wv, c->fb.as<float>(), 0u);
            } else if ((!ops || only_renders) && ns <= ACC_MAX_SAMPLES) {
                hipLaunchKernelGGL(k_accumulate_all, dim3((P + ACC_PIX - 1) / ACC_PIX), dim3(ACC_PIX),
                                   ACC_PIX * (ns + 1) * sizeof(float4), sA, Wv, c->fb.as<float>());
            } else if (!ops) {
                hipLaunchKernelGGL(k_accumulate, dim3((P + 255) / 256), dim3(256), 0, sA, Wv, c->fb.as<float>(), 0u);
            } else {
                // fused frames in call order; a gather between two of them runs on the
                // context stream after the first's accumulate and before the second's
                // (a batch with gathers is one chunk: flush() checks)
                uint32_t fr = 0;
                for (const PendingOp& o : *ops) {
                    if (o.kind == PendingOp::RENDER) {
                        hipLaunchKernelGGL(k_accumulate, dim3((P + 255) / 256), dim3(256), 0, sA, Wv,
                                           c->fb.as<float>(), fr++);
                    } else {
                        hipEvent_t acc = slot_event(f.sync_pool, f.sync_next, true);
                        HIPCHK(hipEventRecord(acc, sA));
                        c->fb_evt = acc;
                        s = op_now(c, o);   // waits fb_evt, sets fb_evt to its own end
                        if (s != KHP_OK) return s;
                        HIPCHK(hipStreamWaitEvent(sA, c->fb_evt, 0));
                    }
                }
            }
            timed(c, f, 3, false, sA);
            if (sB != sA) {  // the next chunk's shadow stages come after this chunk's accumulate
                hipEvent_t acc = slot_event(f.sync_pool, f.sync_next, true);
                HIPCHK(hipEventRecord(acc, sA));
                HIPCHK(hipStreamWaitEvent(sB, acc, 0));
            }
        }
    }
    if (P_all == 0 && ops) {
        // a rank that owns no tile runs no chunk, but its gathers and snapshots
        // still take their place in call order (its peers wait for its gathers)
        for (const PendingOp& o : *ops) {
            if (o.kind == PendingOp::RENDER) continue;
            s = op_now(c, o);
            if (s != KHP_OK) return s;
        }
        if (c->fb_evt) HIPCHK(hipStreamWaitEvent(sA, c->fb_evt, 0));
    }
    if (wa_frames > 1) {
        c->wa.valid = true;
        c->wa.next = *p;
        c->wa.next.first_sample = p->first_sample + p->spp;
        c->wa.gen = c->gen;
        c->wa.Wv = Wv;
        c->wa.nf = wa_frames;
        c->wa.used = 1;
    }
    // join: the batch is done when its last chunk has accumulated
    hipEvent_t e_end = slot_event(f.sync_pool, f.sync_next, true);
    HIPCHK(hipEventRecord(e_end, sA));
    HIPCHK(hipStreamWaitEvent(c->stream, e_end, 0));
    f.done_t = slot_event(f.ev_pool, f.ev_next, false);
    (void)hipEventRecord(f.done_t, c->stream);
    f.done = slot_event(f.sync_pool, f.sync_next, true);
    HIPCHK(hipEventRecord(f.done, c->stream));
    c->fb_evt = f.done;
    f.inflight = true;
    HIPCHK(hipGetLastError());
    if (async) return KHP_OK;
    if (out_rgb && !(p->flags & KHP_RENDER_NO_READBACK)) {
        hipMemcpyKind kind = (p->flags & KHP_RENDER_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        HIPCHK(hipMemcpyAsync(out_rgb, c->fb.p, npix * 3 * sizeof(float), kind, c->stream));
    }
    s = harvest(c, slot);
    if (s != KHP_OK) return s;
    KHPCHK(wait_stream(c, c->stream, "a synchronous frame"));
    if (c->ra.counted) {
        c->st.ahead_finished = c->ra.hst[0];
        c->st.ahead_resumed = c->ra.hst[1];
        c->ra.counted = false;
    }
    c->report_open = false;
    if (sync1) {
        c->series.valid = true;
        c->series.next = *p;
        c->series.next.first_sample = p->first_sample + p->spp;
        c->series.gen = c->gen;
    }
    return KHP_OK;
}


// Frame fusion (asynchronous renders, khp_ctx_params.fuse_frames = n > 1): up to n
// consecutive asynchronous frames with the same geometry, spp, depth and seed
// are enqueued as ONE batch -- one wavefront over all their paths, one
// persistent launch per bounce -- and accumulated one frame after another in
// call order (gathers in between run where they were called).  A launch's
// tail (its slowest ray) is then paid once per batch instead of once per
// frame.  Results are those of the frames rendered one by one.
static bool fusable(const khp_render_params& a, const khp_render_params& b) {
    return a.width == b.width && a.height == b.height && a.spp == b.spp && a.depth == b.depth && a.seed == b.seed &&
           a.tile_size == b.tile_size && a.tile_rank == b.tile_rank && a.tile_nranks == b.tile_nranks &&
           a.flags == b.flags;
}

static khp_status flush(khp_ctx* c) {
    if (c->pend.empty()) return KHP_OK;
    std::vector<PendingOp> ops;
    ops.swap(c->pend);
    const PendingOp* first = nullptr;
    size_t nr = 0;
    bool gathers = false;
    for (const PendingOp& o : ops) {
        if (o.kind == PendingOp::RENDER) {
            if (!first) first = &o;
            ++nr;
        } else {
            gathers = true;
        }
    }
    if (!first) {  // only gathers / snapshots
        for (const PendingOp& o : ops) {
            khp_status s = op_now(c, o);
            if (s != KHP_OK) return s;
        }
        return KHP_OK;
    }
    // a batch with gathers or snapshots must fit one chunk (every frame accumulated
    // before the next frame's gather); otherwise it is split into one-chunk groups
    const uint32_t T = first->p.tile_size ? first->p.tile_size : 64;
    std::vector<uint32_t> tmp;
    size_t P = 0;
    {
        uint32_t nranks = first->p.tile_nranks > 1 ? first->p.tile_nranks : 1;
        uint32_t pkey[5] = {first->p.width, first->p.height, T, nranks > 1 ? first->p.tile_rank : 0u, nranks};
        if (memcmp(pkey, c->pix_key, sizeof(pkey)) == 0 && c->pix.p) {
            P = c->pix_host.size();
        } else {
            owned_pixels(first->p.width, first->p.height, T, nranks > 1 ? first->p.tile_rank : 0u, nranks, tmp);
            P = tmp.size();
        }
    }
    const uint32_t sh_per_path = (c->bd.enabled != 0 && c->S.n_lights > 0) ? c->bd.vertices : 1u;
    const size_t cap_paths = chunk_most(c) / sh_per_path;
    const bool one_chunk = P * (size_t)first->p.spp * nr <= cap_paths;
    if (nr == 1 || !gathers || one_chunk) {
        if (nr == 1) {
            for (const PendingOp& o : ops) {
                khp_status s = o.kind == PendingOp::RENDER ? enqueue_frames(c, &o.p, nullptr, nullptr)
                                                           : op_now(c, o);
                if (s != KHP_OK) return s;
            }
            return KHP_OK;
        }
        return enqueue_frames(c, &first->p, nullptr, &ops);
    }
    // gathers in a batch larger than one chunk: split it into consecutive
    // groups of as many frames as one chunk holds (each with its gathers)
    const size_t per_group = std::max<size_t>(1, cap_paths / std::max<size_t>(1, P * (size_t)first->p.spp));
    std::vector<PendingOp> grp;
    size_t g_r = 0;
    auto run = [&]() -> khp_status {
        khp_status s = KHP_OK;
        if (g_r == 1) {
            for (const PendingOp& o : grp) {
                s = o.kind == PendingOp::RENDER ? enqueue_frames(c, &o.p, nullptr, nullptr) : op_now(c, o);
                if (s != KHP_OK) break;
            }
        } else if (g_r > 1) {
            const PendingOp* f0 = nullptr;
            for (const PendingOp& o : grp)
                if (o.kind == PendingOp::RENDER) { f0 = &o; break; }
            s = enqueue_frames(c, &f0->p, nullptr, &grp);
        } else {
            for (const PendingOp& o : grp) {
                s = op_now(c, o);
                if (s != KHP_OK) break;
            }
        }
        grp.clear();
        g_r = 0;
        return s;
    };
    for (const PendingOp& o : ops) {
        if (o.kind == PendingOp::RENDER && g_r == per_group) {
            khp_status s = run();
            if (s != KHP_OK) return s;
        }
        grp.push_back(o);
        g_r += o.kind == PendingOp::RENDER;
    }
    return run();
}

extern "C" khp_status khp_render(khp_ctx* c, const khp_render_params* p, float* out_rgb) {
    khp_status s = check_params(c, p);
    if (s != KHP_OK) return s;
    HIPCHK(hipSetDevice(c->device));
    const bool stats = (c->flags & KHP_CTX_STATS) != 0 || (p->flags & KHP_RENDER_STATS) != 0;
    const bool async = (p->flags & KHP_RENDER_ASYNC) != 0;
    if (async && (stats || (out_rgb && !(p->flags & KHP_RENDER_NO_READBACK))))
        return fail(KHP_EINVAL, "KHP_RENDER_ASYNC renders take no readback and no instrumentation");
    if (!async) {
        s = flush(c);
        if (s != KHP_OK) return s;
        return enqueue_frames(c, p, out_rgb, nullptr);
    }
    const int fuse = (int)std::max<uint32_t>(1, std::min<uint32_t>(c->prm.fuse_frames, KHP_MAX_FUSE));
    if (fuse <= 1) {
        s = flush(c);
        if (s != KHP_OK) return s;
        return enqueue_frames(c, p, nullptr, nullptr);
    }
    for (const PendingOp& o : c->pend) {
        if (o.kind == PendingOp::RENDER && !fusable(o.p, *p)) {
            s = flush(c);
            if (s != KHP_OK) return s;
            break;
        }
    }
    c->pend.push_back(PendingOp{PendingOp::RENDER, *p, 0});
    size_t nr = 0;
    for (const PendingOp& o : c->pend) nr += o.kind == PendingOp::RENDER;
    if ((int)nr >= fuse) return flush(c);
    return KHP_OK;
}

extern "C" void khp_tonemap_defaults(khp_tonemap* t) {
    if (!t) return;
    *t = khp_tonemap{};
    t->bias = 0.85f;
    t->gamma = 1.0f;
    t->white = 1.0f;
    t->kernel_multiplier = 0.125f;
    t->center_x = t->center_y = -1;
}

// ---- ABI 8: asynchronous 8-bit textures (the GUI's per-pass texture) ----------------------
constexpr size_t KHP_MAX_SNAPS = 64;   // undelivered snapshots; the oldest is waited for beyond this

static Snapshot* find_snap(khp_ctx* c, uint64_t id) {
    for (Snapshot* sn : c->snaps)
        if (sn->id == id) return sn;
    return nullptr;
}

// k_rgba8 on the context stream behind the last framebuffer operation; the next
// framebuffer operation waits for the conversion only, the D2H copy overlaps it.
static khp_status snapshot_now(khp_ctx* c, uint64_t id) {
    Snapshot* sn = find_snap(c, id);
    if (!sn) return fail(KHP_EINVAL, "unknown snapshot");
    if (!c->fb.p) return fail(KHP_ENOTREADY, "nothing rendered yet");
    const uint32_t n = c->fbW * c->fbH;
    if ((size_t)n * 4 != sn->bytes) return fail(KHP_EINVAL, "snapshot size does not match the framebuffer");
    HIPCHK(sn->dbuf.ensure(sn->bytes));
    if (!sn->pinned) HIPCHK(hipHostMalloc((void**)&sn->pinned, sn->bytes, hipHostMallocDefault));
    if (!sn->done) HIPCHK(hipEventCreateWithFlags(&sn->done, hipEventDisableTiming));
    if (!c->snap_evt) HIPCHK(hipEventCreateWithFlags(&c->snap_evt, hipEventDisableTiming));
    if (c->fb_evt) HIPCHK(hipStreamWaitEvent(c->stream, c->fb_evt, 0));
    sn->touched = true;   // from here on the buffers may be in use by the device
    hipLaunchKernelGGL(k_rgba8, dim3((n + 255) / 256), dim3(256), 0, c->stream, c->fb.as<float>(), n,
                       sn->dbuf.as<uint8_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->snap_evt, c->stream));
    c->fb_evt = c->snap_evt;
    HIPCHK(hipMemcpyAsync(sn->pinned, sn->dbuf.p, sn->bytes, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipEventRecord(sn->done, c->stream));
    sn->enqueued = true;
    return KHP_OK;
}

// A snapshot whose conversion or copy was not (completely) enqueued: its ticket is
// removed by id, and its buffers are reused only if nothing was queued on them,
// or once the stream has finished whatever was; if that wait fails
// the snapshot is leaked rather than handed to a later copy still in flight.
static void retire_failed_snapshot(khp_ctx* c, Snapshot* sn) {
    for (size_t i = 0; i < c->snaps.size(); ++i)
        if (c->snaps[i] == sn) {
            c->snaps.erase(c->snaps.begin() + (ptrdiff_t)i);
            break;
        }
    sn->out = nullptr;
    sn->enqueued = false;
    if (sn->touched && wait_stream(c, c->stream, "a failed 8-bit snapshot") != KHP_OK) return;   // leaked
    sn->touched = false;
    c->snap_free.push_back(sn);
}

// Copy completed snapshots with id <= upto into their callers' buffers, oldest first.
// wait: enqueue pending ones (flush) and wait for them; else stop at the first not done.
static khp_status deliver_snapshots(khp_ctx* c, uint64_t upto, bool wait) {
    while (!c->snaps.empty() && c->snaps.front()->id <= upto) {
        Snapshot* sn = c->snaps.front();
        if (!sn->enqueued) {
            if (!wait) return KHP_OK;
            khp_status s = flush(c);
            if (!sn->enqueued) {
                // its conversion never reached the device (an error inside the flush
                // above or an earlier one): drop this ticket only, so later snapshots
                // and syncs still work
                const std::string err = s != KHP_OK ? std::string(khp_last_error())
                                                    : "snapshot " + std::to_string(sn->id) +
                                                          " was not enqueued (an earlier call failed); dropped";
                retire_failed_snapshot(c, sn);
                return fail(s != KHP_OK ? s : KHP_EDEVICE, err);
            }
            if (s != KHP_OK) return s;
        }
        if (wait) {
            KHPCHK(wait_event(c, sn->done, "an 8-bit snapshot"));
        } else {
            const hipError_t q = hipEventQuery(sn->done);
            if (q == hipErrorNotReady) return KHP_OK;
            HIPCHK(q);
        }
        memcpy(sn->out, sn->pinned, sn->bytes);
        c->snaps.erase(c->snaps.begin());
        sn->out = nullptr;
        sn->enqueued = false;
        sn->touched = false;
        c->snap_free.push_back(sn);
    }
    return KHP_OK;
}

extern "C" khp_status khp_read_rgba8_async(khp_ctx* c, uint8_t* out_rgba, uint64_t* ticket) {
    if (!c || !out_rgba || !ticket) return fail(KHP_EINVAL, "null argument");
    HIPCHK(hipSetDevice(c->device));
    uint32_t W = c->fbW, H = c->fbH;  // the frame the snapshot follows: the last pending render, else the framebuffer
    for (const PendingOp& o : c->pend)
        if (o.kind == PendingOp::RENDER) {
            W = o.p.width;
            H = o.p.height;
        }
    if (!W || !H) return fail(KHP_ENOTREADY, "nothing rendered yet");
    if (c->snaps.size() >= KHP_MAX_SNAPS) {
        khp_status s = deliver_snapshots(c, c->snaps.front()->id, true);
        if (s != KHP_OK) return s;
    }
    Snapshot* sn;
    if (!c->snap_free.empty()) {
        sn = c->snap_free.back();
        c->snap_free.pop_back();
    } else {
        sn = new Snapshot();
    }
    const size_t bytes = 4 * (size_t)W * H;
    if (sn->pinned && sn->bytes != bytes) {
        (void)hipHostFree(sn->pinned);
        sn->pinned = nullptr;
    }
    sn->id = c->snap_next++;
    sn->out = out_rgba;
    sn->bytes = bytes;
    sn->enqueued = false;
    c->snaps.push_back(sn);
    *ticket = sn->id;
    if (!c->pend.empty()) {  // behind asynchronous renders waiting for fusion: keep the call order
        PendingOp o{PendingOp::SNAPSHOT, khp_render_params{}, 0, sn->id};
        c->pend.push_back(o);
        return KHP_OK;
    }
    const khp_status st = snapshot_now(c, sn->id);
    if (st != KHP_OK) {  // not (completely) enqueued: the ticket is void
        const std::string err = khp_last_error();
        retire_failed_snapshot(c, sn);
        return fail(st, err);
    }
    return st;
}

extern "C" khp_status khp_snapshot_wait(khp_ctx* c, uint64_t ticket, int wait) {
    if (!c || ticket == 0 || ticket >= c->snap_next) return fail(KHP_EINVAL, "bad snapshot ticket");
    HIPCHK(hipSetDevice(c->device));
    khp_status s = deliver_snapshots(c, ticket, wait != 0);
    if (s != KHP_OK) return s;
    if (find_snap(c, ticket)) return fail(KHP_ENOTREADY, "snapshot not complete yet");
    return KHP_OK;
}

#ifdef KHP_TM_TRACE   // diagnostic builds only: phase times of khp_read_rgba8 to stderr
#define TM_MARK(k) tm_t[k] = std::chrono::steady_clock::now()
#else
#define TM_MARK(k) do { } while (0)
#endif
extern "C" khp_status khp_read_rgba8(khp_ctx* c, const khp_tonemap* tm, uint8_t* out_rgba) {
#ifdef KHP_TM_TRACE
    std::chrono::steady_clock::time_point tm_t[8];
    TM_MARK(0);
#endif
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || !out_rgba) return fail(KHP_EINVAL, "null argument");
    if (!c->fb.p) return fail(KHP_ENOTREADY, "nothing rendered yet");
    HIPCHK(hipSetDevice(c->device));
    const uint32_t n = c->fbW * c->fbH;
    const uint32_t nb = (n + 255) / 256;
    DevMem& out = c->tm_out;
    DevMem &yxy = c->tm_yxy, &bmax = c->tm_bmax, &lgv = c->tm_lgv;
    HIPCHK(out.ensure(4 * (size_t)n));
    if (!tm) {
        hipLaunchKernelGGL(k_rgba8, dim3(nb), dim3(256), 0, c->stream, c->fb.as<float>(), n, out.as<uint8_t>());
    } else {
        HIPCHK(yxy.ensure(12 * (size_t)n));
        HIPCHK(bmax.ensure(4 * (size_t)nb));
        HIPCHK(lgv.ensure(8 * (size_t)n));
        if (c->tm_hl_n < n) {
            if (c->tm_hl) (void)hipHostFree(c->tm_hl);
            c->tm_hl = nullptr;
            c->tm_hl_n = 0;
            HIPCHK(hipHostMalloc((void**)&c->tm_hl, 8 * (size_t)n, hipHostMallocDefault));
            c->tm_hl_n = n;
        }
        if (c->tm_hm_n < nb) {
            if (c->tm_hm) (void)hipHostFree(c->tm_hm);
            c->tm_hm = nullptr;
            c->tm_hm_n = 0;
            HIPCHK(hipHostMalloc((void**)&c->tm_hm, 4 * (size_t)nb, hipHostMallocDefault));
            c->tm_hm_n = nb;
        }
        for (hipEvent_t& e : c->tm_ev)
            if (!e) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        TM_MARK(1);
        hipLaunchKernelGGL(k_tm_yxy, dim3(nb), dim3(256), 0, c->stream, c->fb.as<float>(), n, yxy.as<float>(),
                           bmax.as<float>(), lgv.as<double>());
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(c->tm_hm, bmax.p, 4 * (size_t)nb, hipMemcpyDeviceToHost, c->stream));
        // the log terms come back in chunks, each summed on the host as soon as it has
        // landed, while the next ones are still in flight
        constexpr uint32_t NCH = 16;
        const uint32_t per = (n + NCH - 1) / NCH;
        for (uint32_t ch = 0; ch < NCH; ++ch) {
            const uint32_t a = std::min(n, ch * per), b = std::min(n, a + per);
            if (b > a)
                HIPCHK(hipMemcpyAsync(c->tm_hl + a, lgv.as<double>() + a, 8 * (size_t)(b - a), hipMemcpyDeviceToHost,
                                      c->stream));
            HIPCHK(hipEventRecord(c->tm_ev[ch], c->stream));
        }
        TM_MARK(2);
        float sum = 0.0f;  // RGB_to_Yxy's float running sum, in pixel order (log_sum_feed: bit for bit)
        for (uint32_t ch = 0; ch < NCH; ++ch) {
            // polled, not hipEventSynchronize: a blocking wait per chunk cost ~0.15 ms of
            // wake-up each (2.4 ms per texture, profiles/r05e_tonemap_trace.txt)
            if (bounded_waits(c)) {
                KHPCHK(wait_event(c, c->tm_ev[ch], "the 8-bit texture's log luminances"));
            } else {
                // spin briefly (a chunk usually lands within ~0.1 ms), then yield, then
                // block: no core burnt for a long copy, no endless spin on a hung device
                for (int spins = 0;; ++spins) {
                    const hipError_t q = hipEventQuery(c->tm_ev[ch]);
                    if (q == hipSuccess) break;
                    if (q != hipErrorNotReady) HIPCHK(q);
                    if (spins >= 4096) {
                        HIPCHK(hipEventSynchronize(c->tm_ev[ch]));
                        break;
                    }
                    if (spins >= 256) std::this_thread::yield();
                }
            }
            const uint32_t a = std::min(n, ch * per), b = std::min(n, a + per);
            sum = log_sum_feed(sum, c->tm_hl + a, b - a);
#ifdef KHP_TM_TRACE
            if (ch == 0) TM_MARK(3);
#endif
        }
        TM_MARK(4);
        const float* hm = c->tm_hm;
        float mx = 1e-06f;
        for (uint32_t b = 0; b < nb; ++b) mx = (mx < hm[b]) ? hm[b] : mx;
        // Tonemapper::map / tonemapping scalars, in KIRK's float/double mix
        float world_lum = sum / (float)n;
        if (tm->center_weight) {
            // window and mask on the host, as Tonemapping.cpp:186-236 builds them
            const int width = (int)c->fbW, height = (int)c->fbH;
            const int cx = tm->center_x < 0 ? width / 2 : tm->center_x;
            const int cy = tm->center_y < 0 ? height / 2 : tm->center_y;
            int ks = width < height ? (int)(width * tm->kernel_multiplier) : (int)(height * tm->kernel_multiplier);
            if (ks > width || ks > height) ks = std::min(width, height);
            else if (ks < 1) ks = 1;
            if (ks % 2 == 0) ks -= 1;
            const int half = (int)std::floor(ks * 0.5);
            const int xs = cx + half > width ? width - ks : (cx - half < 0 ? 0 : cx - half);
            const int ys = cy + half > height ? height - ks : (cy - half < 0 ? 0 : cy - half);
            if ((long)(xs + ks) * (ys + ks) > (long)width * height || xs < 0 || ys < 0)
                return fail(KHP_EINVAL, "tonemap center window reads outside the image");
            std::vector<double> mask((size_t)ks * ks);
            double acc = 0.0;
            for (int idx = 0; idx < ks * ks; ++idx) {
                const int x = idx % ks - half, y = idx / ks - half;
                const float r = (float)std::sqrt((double)(x * x + y * y));
                mask[idx] = std::exp(-std::log(2.0) * std::pow((double)(r / (float)half), 2.0));
            }
            for (double m : mask) acc += m;
            const double mean = (double)(ks * ks) / acc;
            const uint32_t nbc = (uint32_t)(ks * ks + 255) / 256;
            DevMem dmask, cterm;
            HIPCHK(dmask.ensure(mask.size() * 8));
            HIPCHK(cterm.ensure(8 * (size_t)ks * ks));
            HIPCHK(hipMemcpyAsync(dmask.p, mask.data(), mask.size() * 8, hipMemcpyHostToDevice, c->stream));
            hipLaunchKernelGGL(k_tm_center, dim3(nbc), dim3(256), 0, c->stream, yxy.as<float>(), ks, xs, ys,
                               dmask.as<double>(), mean, cterm.as<double>());
            std::vector<double> hc((size_t)ks * ks);
            HIPCHK(hipMemcpyAsync(hc.data(), cterm.p, 8 * hc.size(), hipMemcpyDeviceToHost, c->stream));
            KHPCHK(wait_stream(c, c->stream, "the 8-bit texture"));
            double cs = 0.0;  // luminance_from_center's double running sum, in its loop order
            for (double v : hc) cs += v;
            world_lum = (float)(cs / (ks * ks));
        }
        TmScalars t{};
        t.exposure = (float)pow(2.0, (double)tm->exposure);
        t.av_lum = expf(world_lum) / 1.0f;
        t.biasP = logf(tm->bias) / -0.693147f;
        t.contP = 1.0f / tm->contrast;
        t.contrast_on = tm->contrast != 0.0f;
        t.Lmax = mx / t.av_lum;
        t.divider = log10f(t.Lmax + 1.0f);
        t.gamma_on = (double)tm->gamma != 1.0;
        t.rec = tm->rec_gamma != 0;
        if (t.rec) {
            t.inv_gamma = (float)(0.45 / (double)tm->gamma * 2.0);
            t.slope = 4.5f;
            t.start = 0.018f;
            if ((double)tm->gamma >= 2.1) {
                t.start = (float)(0.018 / ((double)(tm->gamma - 2.0f) * 7.5));
                t.slope = (float)(4.5 * ((double)(tm->gamma - 2.0f) * 7.5));
            } else if ((double)tm->gamma <= 1.9) {
                t.start = (float)(0.018 * ((double)(2.0f - tm->gamma) * 7.5));
                t.slope = (float)(4.5 / ((double)(2.0f - tm->gamma) * 7.5));
            }
        } else {
            t.inv_gamma = 1.0f / tm->gamma;
        }
        t.clamp_on = tm->white != 1.0f || tm->black != 0.0f;
        t.white = tm->white;
        t.black = tm->black;
        hipLaunchKernelGGL(k_tm_map, dim3(nb), dim3(256), 0, c->stream, yxy.as<float>(), n, t, out.as<uint8_t>());
        TM_MARK(5);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out_rgba, out.p, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    KHPCHK(wait_stream(c, c->stream, "the 8-bit texture"));
#ifdef KHP_TM_TRACE
    TM_MARK(6);
    if (tm) {
        auto d = [&](int a, int b) { return std::chrono::duration<double, std::milli>(tm_t[b] - tm_t[a]).count(); };
        fprintf(stderr, "[khp tm] setup %.3f enqueue %.3f first-chunk %.3f sum %.3f map-enqueue %.3f out %.3f total %.3f ms\n",
                d(0, 1), d(1, 2), d(2, 3), d(3, 4), d(4, 5), d(5, 6), d(0, 6));
    }
#endif
    return KHP_OK;
}


extern "C" khp_status khp_read_bvh(khp_ctx* c, uint32_t* n_nodes, uint32_t* depth, float* node_boxes,
                                   int32_t* node_first, int32_t* node_count, int32_t* object_ids) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || !n_nodes) return fail(KHP_EINVAL, "ctx or n_nodes is null");
    if (!c->built) return fail(KHP_ENOTREADY, "khp_build_accel first");
    HostScene& hs = c->hs;
    if (c->tree_on_device && hs.nodes.size() != c->tree.n_nodes) {
        HIPCHK(hipSetDevice(c->device));
        std::string err = download_tree(c->tree, hs, c->stream);
        if (!err.empty()) return fail(KHP_EDEVICE, err);
    }
    *n_nodes = (uint32_t)hs.nodes.size();
    if (depth) *depth = hs.depth;
    for (size_t i = 0; i < hs.nodes.size(); ++i) {
        const BuildNode& n = hs.nodes[i];
        if (node_boxes) {
            const float b[6] = {n.mn.x, n.mn.y, n.mn.z, n.mx.x, n.mx.y, n.mx.z};
            memcpy(node_boxes + 6 * i, b, sizeof(b));
        }
        if (node_first) node_first[i] = n.count ? n.first : -1;
        if (node_count) node_count[i] = n.count;
    }
    if (object_ids)
        for (uint32_t i = 0; i < hs.n_obj; ++i) object_ids[i] = (int32_t)hs.ids[i];
    return KHP_OK;
}


extern "C" khp_status khp_read_layout(khp_ctx* c, uint32_t* n_records, uint32_t* n_slots, void* node_records,
                                      float* prim_records, uint32_t* prim_aux) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || !n_records || !n_slots) return fail(KHP_EINVAL, "null argument");
    if (!c->built) return fail(KHP_ENOTREADY, "khp_build_accel first");
    HIPCHK(hipSetDevice(c->device));
    *n_records = c->n_dnodes;
    *n_slots = c->n_slots;
    if (node_records && c->n_dnodes)
        HIPCHK(hipMemcpyAsync(node_records, c->nodes.p, sizeof(DevNode) * (size_t)c->n_dnodes, hipMemcpyDeviceToHost,
                              c->stream));
    if (prim_records && c->n_slots)
        HIPCHK(hipMemcpyAsync(prim_records, c->prims.p, 64 * (size_t)c->n_slots, hipMemcpyDeviceToHost, c->stream));
    if (prim_aux && c->n_slots)
        HIPCHK(hipMemcpyAsync(prim_aux, c->aux.p, sizeof(Aux) * (size_t)c->n_slots, hipMemcpyDeviceToHost, c->stream));
    KHPCHK(wait_stream(c, c->stream, "the layout read"));
    return KHP_OK;
}

extern "C" khp_status khp_debug_shadow_queue(khp_ctx* c, uint32_t* n, float* orig, float* dir, float* tmax) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || !n) return fail(KHP_EINVAL, "null argument");
    const uint32_t m = (uint32_t)(c->dump_sh.size() / 7);
    if (orig && dir && tmax) {
        for (uint32_t i = 0; i < m && i < *n; ++i) {
            const float* v = c->dump_sh.data() + 7 * (size_t)i;
            for (int k = 0; k < 3; ++k) {
                orig[3 * (size_t)i + k] = v[k];
                dir[3 * (size_t)i + k] = v[3 + k];
            }
            tmax[i] = v[6];
        }
    }
    *n = m;
    return KHP_OK;
}

extern "C" khp_status khp_debug_queue(khp_ctx* c, uint32_t* n, float* orig, float* dir) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || !n) return fail(KHP_EINVAL, "null argument");
    const uint32_t m = (uint32_t)(c->dump.size() / 6);
    if (orig && dir) {
        for (uint32_t i = 0; i < m && i < *n; ++i)
            for (int k = 0; k < 3; ++k) {
                orig[3 * (size_t)i + k] = c->dump[(size_t)k * m + i];
                dir[3 * (size_t)i + k] = c->dump[(size_t)(3 + k) * m + i];
            }
    }
    *n = m;
    return KHP_OK;
}

extern "C" khp_status khp_read_framebuffer(khp_ctx* c, float* out_rgb) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || !out_rgb) return fail(KHP_EINVAL, "null argument");
    if (!c->fb.p) return fail(KHP_ENOTREADY, "nothing rendered yet");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(out_rgb, c->fb.p, (size_t)c->fbW * c->fbH * 3 * sizeof(float), hipMemcpyDeviceToHost,
                          c->stream));
    KHPCHK(wait_stream(c, c->stream, "the framebuffer read"));
    return KHP_OK;
}

// ---- batch queries through the persistent wavefront kernels (test hook) -------------
// khp_ctx_params.trace_kernels = 1|2 routes khp_trace_closest / khp_trace_any through k_extend /
// k_shadow -- the kernels the renderer uses -- instead of the one-ray-per-thread
// kernels, so tests can check the production traversal ray by ray.
__global__ void k_load_rays(uint32_t n, const float* orig, const float* dir, Wave Wv, int as_shadow,
                            const float* tmax) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {
        Wv.cnt->nq[0] = as_shadow ? 0u : n;
        Wv.shq->nsh = as_shadow ? n : 0u;
    }
    if (i >= n) return;
    Ray r = make_ray(ld3(orig + 3 * (size_t)i), ld3(dir + 3 * (size_t)i));
    if (as_shadow) {
        Wv.sh[Wv.shs * (size_t)i] = make_float4(r.o.x, r.o.y, r.o.z, tmax[i]);
        Wv.sh[Wv.shs * (size_t)i + 1] = make_float4(r.d.x, r.d.y, r.d.z, 0.0f);
    } else {
        Wv.qo[0][0][i] = r.o.x; Wv.qo[0][1][i] = r.o.y; Wv.qo[0][2][i] = r.o.z;
        Wv.qd[0][0][i] = r.d.x; Wv.qd[0][1][i] = r.d.y; Wv.qd[0][2][i] = r.d.z;
    }
}

__global__ void k_store_hits(DevScene S, uint32_t n, Wave Wv, float* t, int32_t* obj, float* uv) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t sl = Wv.hslot[i];
    t[i] = Wv.ht[i];
    obj[i] = sl >= 0 ? (int32_t)S.aux[sl].obj : -1;
    float u = 0.0f, v = 0.0f;  // the traversal keeps t and slot; barycentrics of a triangle hit from the ray
    if (sl >= 0) {
        const float4* p = S.prims + 4 * (size_t)sl;
        if (is_tri(p[0])) {
            Ray r;
            r.o = mk(Wv.qo[0][0][i], Wv.qo[0][1][i], Wv.qo[0][2][i]);
            r.d = mk(Wv.qd[0][0][i], Wv.qd[0][1][i], Wv.qd[0][2][i]);
            tri_uv(p[0], p[1], p[2], r, u, v);
        }
    }
    uv[2 * i] = u;
    uv[2 * i + 1] = v;
}

// prm.trace_kernels -- 0: one-ray-per-thread kernels; 1: instrumented
// persistent kernels (KIRK's visit counts); 2: production persistent kernels.
static int trace_persistent(const khp_ctx* c) { return (int)c->prm.trace_kernels; }

static khp_status trace_persistent_run(khp_ctx* c, uint32_t n, const float* orig, const float* dir,
                                       const float* tmax_h, float* t_out, int32_t* obj_out, float* uv_out,
                                       uint8_t* hit_out) {
    const bool shadow = hit_out != nullptr;
    PathSet& w = c->ps[0];
    c->wa.valid = false;   // the batch query API reuses ps[0]
    khp_status s = ensure_wave(c, w, n);
    if (s != KHP_OK) return s;
    DevMem o, d, tm, t, ob, uv;
    HIPCHK(upload(o, orig, 3 * (size_t)n, c->stream));
    HIPCHK(upload(d, dir, 3 * (size_t)n, c->stream));
    if (shadow) HIPCHK(upload(tm, tmax_h, (size_t)n, c->stream));
    HIPCHK(hipMemsetAsync(w.cnt.p, 0, sizeof(Counters), c->stream));
    HIPCHK(hipMemsetAsync(w.shqb.p, 0, 2 * sizeof(ShadowQ), c->stream));
    Wave Wv = wave_view(c, w);
    hipLaunchKernelGGL(k_load_rays, dim3((n + 255) / 256), dim3(256), 0, c->stream, n, o.as<float>(), d.as<float>(),
                       Wv, shadow ? 1 : 0, tm.as<float>());
    const bool prod = trace_persistent(c) == 2;
    hipEvent_t e0 = next_event(c), e1 = next_event(c);
    (void)hipEventRecord(e0, c->stream);
    if (shadow) {
        SpillArea sp{w.spill_sh.as<int4>(), (uint32_t)c->grid_sh * TRAV_BLOCK};
        const bool wide = c->S.wide != nullptr && c->prm.wide_from == 0;  // the two-level any-hit loop ray by ray
        launch_shadow(!prod, wide, wide ? c->grid_sh_w : c->grid_sh, c->stream, c->S, Wv, sp);
        (void)hipEventRecord(e1, c->stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(hit_out, Wv.vis, n, hipMemcpyDeviceToHost, c->stream));
    } else {
        SpillArea sp{w.spill.as<int4>(), (uint32_t)c->grid_ext_max * TRAV_BLOCK};
        const bool wide = c->S.wide != nullptr && c->prm.wide_from == 0;  // the two-level loop ray by ray
        launch_extend(!prod, false, wide, wide ? c->grid_ext_w : c->grid_ext, c->stream, c->S, Wv, 0, sp);
        (void)hipEventRecord(e1, c->stream);
        HIPCHK(t.ensure(4 * (size_t)n));
        HIPCHK(ob.ensure(4 * (size_t)n));
        HIPCHK(uv.ensure(8 * (size_t)n));
        hipLaunchKernelGGL(k_store_hits, dim3((n + 255) / 256), dim3(256), 0, c->stream, c->S, n, Wv, t.as<float>(),
                           ob.as<int32_t>(), uv.as<float>());
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(t_out, t.p, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(obj_out, ob.p, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
        if (uv_out) HIPCHK(hipMemcpyAsync(uv_out, uv.p, 8 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    }
    Counters hc;
    HIPCHK(hipMemcpyAsync(&hc, w.cnt.p, sizeof(hc), hipMemcpyDeviceToHost, c->stream));
    KHPCHK(wait_stream(c, c->stream, "the ray queries"));
    c->st.node_visits = shadow ? hc.sh_node_visits : hc.node_visits;
    c->st.prim_tests = shadow ? hc.sh_prim_tests : hc.prim_tests;
    c->st.stack_spills = hc.spills;
    float kms = 0.0f;
    (void)hipEventElapsedTime(&kms, e0, e1);
    c->st.render_ms = kms;  // persistent query: traversal kernel time
    c->ev_next = 0;
    return KHP_OK;
}

extern "C" khp_status khp_trace_closest(khp_ctx* c, uint32_t n, const float* orig, const float* dir, float* t_out,
                                        int32_t* obj_out, float* uv_out) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || (n && (!orig || !dir || !t_out || !obj_out))) return fail(KHP_EINVAL, "null argument");
    if (!c->built) return fail(KHP_ENOTREADY, "khp_build_accel first");
    if (n == 0) return KHP_OK;
    HIPCHK(hipSetDevice(c->device));
    if (trace_persistent(c)) return trace_persistent_run(c, n, orig, dir, nullptr, t_out, obj_out, uv_out, nullptr);
    DevMem o, d, t, ob, uv, stb;
    HIPCHK(upload(o, orig, 3 * (size_t)n, c->stream));
    HIPCHK(upload(d, dir, 3 * (size_t)n, c->stream));
    HIPCHK(t.ensure(4 * (size_t)n));
    HIPCHK(ob.ensure(4 * (size_t)n));
    HIPCHK(uv.ensure(8 * (size_t)n));
    HIPCHK(stb.ensure(16));
    HIPCHK(hipMemsetAsync(stb.p, 0, 16, c->stream));
    hipLaunchKernelGGL(k_trace_closest<true>, dim3((n + 255) / 256), dim3(256), 0, c->stream, c->S, n,
                       o.as<float>(), d.as<float>(), t.as<float>(), ob.as<int32_t>(), uv.as<float>(),
                       stb.as<unsigned long long>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(t_out, t.p, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(obj_out, ob.p, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    if (uv_out) HIPCHK(hipMemcpyAsync(uv_out, uv.p, 8 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    unsigned long long sv[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(sv, stb.p, 16, hipMemcpyDeviceToHost, c->stream));
    KHPCHK(wait_stream(c, c->stream, "the ray queries"));
    c->st.node_visits = sv[0];
    c->st.prim_tests = sv[1];
    return KHP_OK;
}

extern "C" khp_status khp_trace_any(khp_ctx* c, uint32_t n, const float* orig, const float* dir, const float* tmax,
                                    uint8_t* hit_out) {
    if (c) {  // complete asynchronous frames first
        khp_status dr = drain(c);
        if (dr != KHP_OK) return dr;
    }
    if (!c || (n && (!orig || !dir || !tmax || !hit_out))) return fail(KHP_EINVAL, "null argument");
    if (!c->built) return fail(KHP_ENOTREADY, "khp_build_accel first");
    if (n == 0) return KHP_OK;
    HIPCHK(hipSetDevice(c->device));
    if (trace_persistent(c)) return trace_persistent_run(c, n, orig, dir, tmax, nullptr, nullptr, nullptr, hit_out);
    DevMem o, d, tm, h;
    HIPCHK(upload(o, orig, 3 * (size_t)n, c->stream));
    HIPCHK(upload(d, dir, 3 * (size_t)n, c->stream));
    HIPCHK(upload(tm, tmax, (size_t)n, c->stream));
    HIPCHK(h.ensure((size_t)n));
    hipLaunchKernelGGL(k_trace_any, dim3((n + 255) / 256), dim3(256), 0, c->stream, c->S, n, o.as<float>(),
                       d.as<float>(), tm.as<float>(), h.as<uint8_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(hit_out, h.p, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    KHPCHK(wait_stream(c, c->stream, "the ray queries"));
    return KHP_OK;
}

extern "C" khp_status khp_get_stats(khp_ctx* c, khp_stats* out) {
    if (!c || !out) return fail(KHP_EINVAL, "null argument");
    *out = c->st;
    return KHP_OK;
}

#ifdef KHP_PATH_PROFILE
// Diagnostic builds only (not part of the ABI): copies the k_path per-wave
// records written since the last call (6 x u64 each, see g_wprof) and resets them.
extern "C" khp_status khp_debug_wave_profile(khp_ctx* c, unsigned long long* out, uint32_t max_waves, uint32_t* n) {
    if (!c || !out || !n) return fail(KHP_EINVAL, "null argument");
    KHPCHK(drain(c));
    HIPCHK(hipSetDevice(c->device));
    uint32_t cnt = 0;
    HIPCHK(hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(g_wprof_n), sizeof(cnt)));
    cnt = std::min<uint32_t>(std::min<uint32_t>(cnt, KHP_WPROF_MAX), max_waves);
    if (cnt) HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wprof), 6 * sizeof(unsigned long long) * cnt));
    const uint32_t zero = 0;
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_wprof_n), &zero, sizeof(zero)));
    *n = cnt;
    return KHP_OK;
}
// render-ahead timeline of the last launch: the 100 MHz clock when its last own path
// ended and when the first wave saw that (~0ull: none); read and reset
extern "C" khp_status khp_debug_ahead_profile(khp_ctx* c, unsigned long long* out) {
    if (!c || !out) return fail(KHP_EINVAL, "null argument");
    KHPCHK(drain(c));
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ra_prof), 2 * sizeof(unsigned long long)));
    const unsigned long long init[2] = {0ull, ~0ull};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_ra_prof), init, sizeof(init)));
    return KHP_OK;
}
#endif

// ---- RCCL ---------------------------------------------------------------------------------
// The communicator is non-blocking (ncclConfig_t.blocking = 0, ABI 11): an RCCL call
// may return ncclInProgress while RCCL finishes it in the background, and the
// communicator must not be used, nor anything enqueued behind the call on its
// stream, until ncclCommGetAsyncError reports ncclSuccess.  comm_settle does
// that poll with the context's bound, so no init, send, receive or group end can
// hang the caller: a timeout or an error aborts the communicator (ncclCommAbort)
// and returns KHP_EDEVICE naming this rank and its peers.
static khp_status comm_settle(khp_ctx* c, ncclResult_t r, const std::string& what) {
    if (!c->comm) return fail(KHP_EDEVICE, comm_who(c) + ": " + what + ": no communicator");
    const auto t0 = std::chrono::steady_clock::now();
    COMM_TRACE("settle %s: r=%d", what.c_str(), (int)r);
    for (int spins = 0; r == ncclInProgress; ++spins) {
        ncclResult_t ae = ncclInProgress;
        const ncclResult_t q = ncclCommGetAsyncError(c->comm, &ae);
        r = q != ncclSuccess ? q : ae;
        if (r != ncclInProgress) break;
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms > c->comm_timeout_ms)
            return comm_abort(c, comm_who(c) + ": " + what + " did not complete within " +
                                     std::to_string(c->comm_timeout_ms) + " ms (peers not joined or not progressing); "
                                     "communicator aborted");
        if (spins < 256) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    COMM_TRACE("settled %s: r=%d", what.c_str(), (int)r);
    if (r != ncclSuccess)
        return comm_abort(c, comm_who(c) + ": " + what + ": " + ncclGetErrorString(r) + "; communicator aborted");
    return KHP_OK;
}

// Frees the communicator: finalize (flushes issued operations; bounded), then
// destroy; a finalize that does not settle aborts instead.
static void comm_release(khp_ctx* c) {
    if (c->comm && comm_settle(c, ncclCommFinalize(c->comm), "ncclCommFinalize") == KHP_OK && c->comm)
        (void)ncclCommDestroy(c->comm);
    c->comm = nullptr;
    c->comm_job.reset();
    // also after an abort (comm already null): the dead communicator's state
    // must not keep the next group's or the local group's waits polling
    c->comm_dead.clear();
    for (const khp_ctx::CommOp& op : c->comm_ops)
        for (hipEvent_t e : {op.pre, op.post})
            if (e) (void)hipEventDestroy(e);
    c->comm_ops.clear();
    for (hipEvent_t e : c->comm_evt_free) (void)hipEventDestroy(e);
    c->comm_evt_free.clear();
}

extern "C" khp_status khp_comm_unique_id(uint8_t out_id[128]) {
    if (!out_id) return fail(KHP_EINVAL, "null argument");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(KHP_EDEVICE, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    memcpy(out_id, &id, 128);
    return KHP_OK;
}

extern "C" khp_status khp_comm_set_timeout(khp_ctx* c, uint32_t timeout_ms) {
    if (!c || timeout_ms == 0) return fail(KHP_EINVAL, "khp_comm_set_timeout: null context or zero timeout");
    c->comm_timeout_ms = timeout_ms;
    return KHP_OK;
}

// khp_debug_comm_wait's gate: one wave spins (sleeping) until the host sets *flag,
// or for at most max_ticks of the 100 MHz clock, so it always ends.
__global__ void k_gate(const volatile uint32_t* flag, unsigned long long max_ticks) {
    const unsigned long long t0 = wall_clock64();
    while (*flag == 0u && wall_clock64() - t0 < max_ticks) __builtin_amdgcn_s_sleep(64);
}

extern "C" khp_status khp_debug_comm_wait(khp_ctx* c, int scenario, uint32_t bound_ms, uint32_t release_ms,
                                          double* waited_ms) {
    if (!c || !waited_ms || scenario < 0 || scenario > 2 || bound_ms == 0) return fail(KHP_EINVAL, "bad arguments");
    if (c->comm) return fail(KHP_EINVAL, "khp_debug_comm_wait: the context has a communicator");
    HIPCHK(hipSetDevice(c->device));
    KHPCHK(drain(c));
    uint32_t* flag = nullptr;
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&flag), sizeof(uint32_t), hipHostMallocCoherent));
    *flag = 0u;
    const std::string dead_before = c->comm_dead;
    const uint32_t bound_before = c->comm_timeout_ms;
    c->comm_dead = "khp_debug_comm_wait";   // waits are bounded as after a communicator's abort
    c->comm_timeout_ms = bound_ms;
    auto gate = [&]() { hipLaunchKernelGGL(k_gate, dim3(1), dim3(64), 0, c->stream, flag, 1000000000ull); };
    hipError_t e = hipSuccess;
    if (scenario == 0) {
        gate();
        e = comm_op_begin(c);
        if (e == hipSuccess) e = comm_op_end(c);
    } else if (scenario == 1) {
        e = comm_op_begin(c);
        gate();
        if (e == hipSuccess) e = comm_op_end(c);
    } else {
        e = comm_op_begin(c);
        gate();
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::thread rel([flag, release_ms] {
        std::this_thread::sleep_for(std::chrono::milliseconds(release_ms));
        __atomic_store_n(flag, 1u, __ATOMIC_RELEASE);
    });
    khp_status st = e == hipSuccess ? wait_stream(c, c->stream, "the test gate")
                                    : fail(KHP_EDEVICE, std::string("hipEventRecord: ") + hipGetErrorString(e));
    *waited_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    const std::string msg = st == KHP_OK ? std::string() : last_error();
    rel.join();
    (void)hipStreamSynchronize(c->stream);   // the gate has ended (released)
    while (comm_op_pending(c)) {}            // every bracket completed: retire them
    c->comm_ops.clear();
    c->comm_dead = dead_before;
    c->comm_timeout_ms = bound_before;
    (void)hipHostFree(flag);
    if (st != KHP_OK) return fail(st, msg);
    return KHP_OK;
}

static void leave_local_group(khp_ctx* c) {
    if (c->lgroup)
        for (auto& m : *c->lgroup)
            if (m == c) m = nullptr;
    c->lgroup.reset();
    c->lg_seq = 0;
    for (size_t k = 0; k < LG_SLOTS; ++k) {
        c->lg_stamp[k] = 0;
        c->lg_taken[k] = false;
        c->lg_count[k] = 0;
    }
}

// RCCL's ncclCommInitRankConfig does not return while a peer is missing, even
// for a non-blocking communicator (measured on this image, RCCL 2.27.7: it stays
// in its bootstrap, profiles/r04d_comm_probe.log).  The call therefore runs on
// a helper thread and the caller waits for it with the context's bound; on a
// timeout the caller returns KHP_EDEVICE and the thread is left to finish
// alone: if the init ever completes it aborts the communicator nobody waits
// for, otherwise it stays blocked until the process exits.
struct CommInitJob {
    std::mutex m;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclSuccess;
    // A non-blocking init goes on in RCCL's background job after the call
    // returns, and may still read its arguments: they live here, with the job.
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    ncclUniqueId uid;
};

extern "C" khp_status khp_comm_init(khp_ctx* c, int nranks, int rank, const uint8_t id[128]) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(KHP_EINVAL, "bad comm arguments");
    HIPCHK(hipSetDevice(c->device));
    KHPCHK(drain(c));   // complete asynchronous frames (and gathers) first
    comm_release(c);
    leave_local_group(c);
    memset(c->gather_key, 0, sizeof(c->gather_key));
    c->nranks = nranks;
    c->rank = rank;
    ncclUniqueId uid;
    memcpy(&uid, id, 128);
    auto job = std::make_shared<CommInitJob>();
    const int device = c->device;
    try {
        job->uid = uid;
        job->cfg.blocking = 0;   // every later RCCL call is polled with the context's bound (comm_settle)
        std::thread([job, nranks, rank, device]() {
            (void)hipSetDevice(device);
            ncclComm_t comm = nullptr;
            COMM_TRACE("ncclCommInitRankConfig begin (rank %d of %d)", rank, nranks);
            ncclResult_t r = ncclCommInitRankConfig(&comm, nranks, job->uid, rank, &job->cfg);
            COMM_TRACE("ncclCommInitRankConfig returned %d", (int)r);
            // the init completes here, on this thread, before the communicator is handed over
            while (r == ncclInProgress && comm) {
                ncclResult_t ae = ncclInProgress;
                const ncclResult_t q = ncclCommGetAsyncError(comm, &ae);
                r = q != ncclSuccess ? q : ae;
                if (r != ncclInProgress) break;
                {
                    std::lock_guard<std::mutex> lk(job->m);
                    if (job->abandoned) break;
                }
                std::this_thread::sleep_for(std::chrono::microseconds(200));
            }
            COMM_TRACE("init settled %d", (int)r);
            std::lock_guard<std::mutex> lk(job->m);
            if (job->abandoned) {   // the caller gave up: nobody will use this communicator
                if (comm) (void)ncclCommAbort(comm);
                return;
            }
            job->comm = comm;
            job->r = r;
            job->done = true;
            job->cv.notify_all();
        }).detach();
    } catch (const std::exception& e) {
        return fail(KHP_EDEVICE, std::string("khp_comm_init: cannot start the init thread: ") + e.what());
    }
    {
        std::unique_lock<std::mutex> lk(job->m);
        if (!job->cv.wait_for(lk, std::chrono::milliseconds(c->comm_timeout_ms), [&] { return job->done; })) {
            job->abandoned = true;
            return fail(KHP_EDEVICE, comm_who(c) + ": RCCL communicator init did not return within " +
                                         std::to_string(c->comm_timeout_ms) +
                                         " ms (a peer never joined); this context has no communicator");
        }
    }
    const ncclResult_t r = job->r;
    if (r != ncclSuccess && r != ncclInProgress) {
        if (job->comm) (void)ncclCommAbort(job->comm);
        return fail(KHP_EDEVICE, comm_who(c) + ": ncclCommInitRankConfig: " + ncclGetErrorString(r));
    }
    c->comm = job->comm;
    c->comm_job = job;
    const khp_status s = comm_settle(c, r, "RCCL communicator init");   // r is ncclSuccess here
    if (s != KHP_OK) c->comm_dead.clear();   // nothing was enqueued on the comm: the context stays usable
    return s;
}

extern "C" khp_status khp_comm_init_local(khp_ctx* const* ctxs, int nranks) {
    if (!ctxs || nranks < 1) return fail(KHP_EINVAL, "bad local group");
    for (int r = 0; r < nranks; ++r) {
        if (!ctxs[r]) return fail(KHP_EINVAL, "null context in local group");
        if (ctxs[r]->device != ctxs[0]->device)
            return fail(KHP_EINVAL, "local group: every context must be on the same device");
        for (int q = 0; q < r; ++q)
            if (ctxs[q] == ctxs[r]) return fail(KHP_EINVAL, "local group: a context appears twice");
    }
    for (int r = 0; r < nranks; ++r) {
        khp_ctx* c = ctxs[r];
        HIPCHK(hipSetDevice(c->device));
        KHPCHK(drain(c));
    }
    auto g = std::make_shared<std::vector<khp_ctx*>>(ctxs, ctxs + nranks);
    for (int r = 0; r < nranks; ++r) {
        khp_ctx* c = ctxs[r];
        comm_release(c);
        leave_local_group(c);   // stamps cleared: nothing packed for an earlier group is ever copied
        c->lgroup = g;
        c->nranks = nranks;
        c->rank = r;
        memset(c->gather_key, 0, sizeof(c->gather_key));
    }
    return KHP_OK;
}

extern "C" khp_status khp_gather_framebuffer(khp_ctx* c, const khp_render_params* p, int root) {
    khp_status s = check_params(c, p);
    if (s != KHP_OK) return s;
    if (!c->comm && !c->lgroup)
        return fail(KHP_ENOTREADY, c->comm_dead.empty() ? std::string("khp_comm_init first")
                                                        : "the communicator was aborted (" + c->comm_dead +
                                                              "); khp_comm_init again");
    if (root < 0 || root >= c->nranks) return fail(KHP_EINVAL, "bad root");
    if (p->tile_nranks != (uint32_t)c->nranks) return fail(KHP_EINVAL, "tile_nranks must equal the comm size");
    if (!c->pend.empty()) {  // behind asynchronous renders waiting for fusion: keep the call order
        c->pend.push_back(PendingOp{PendingOp::GATHER, *p, root});
        return KHP_OK;
    }
    return gather_now(c, p, root);
}

// In-process group transport (khp_comm_init_local).  Sender: pack into slot
// seq % LG_SLOTS once the root has taken the slot's previous content, stamp it
// with seq.  Root: every sender's slot must carry this gather's stamp (else
// KHP_ENOTREADY, nothing enqueued, the root's sequence unchanged); copy each,
// and record the sender's "copied" event behind the copy so the sender's next
// pack into that slot waits for it.
static khp_status local_send(khp_ctx* c, uint32_t P) {
    const uint64_t seq = c->lg_seq;
    const size_t k = seq % LG_SLOTS;
    if (c->lg_stamp[k] && !c->lg_taken[k])
        return fail(KHP_ENOTREADY, "local group: " + comm_who(c) + " is " + std::to_string(LG_SLOTS) +
                                       " gathers ahead of the root (gather " + std::to_string(c->lg_stamp[k] - 1) +
                                       " in ring slot " + std::to_string(k) + " not taken yet)");
    HIPCHK(c->lg_slots[k].ensure((size_t)P * 3 * sizeof(float) + 16));
    if (!c->lg_evts[k]) HIPCHK(hipEventCreateWithFlags(&c->lg_evts[k], hipEventDisableTiming));
    if (!c->lg_copied[k]) HIPCHK(hipEventCreateWithFlags(&c->lg_copied[k], hipEventDisableTiming));
    if (c->lg_stamp[k]) HIPCHK(hipStreamWaitEvent(c->stream, c->lg_copied[k], 0));  // the root's copy of the old content
    if (P) hipLaunchKernelGGL(k_pack, dim3((P + 255) / 256), dim3(256), 0, c->stream, c->fb.as<float>(),
                              c->stage_pix.as<uint32_t>(), P, c->lg_slots[k].as<float>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->lg_evts[k], c->stream));
    c->lg_stamp[k] = seq + 1;
    c->lg_taken[k] = false;
    c->lg_count[k] = P;
    c->lg_seq = seq + 1;
    return KHP_OK;
}

static khp_status local_receive(khp_ctx* c, int root, size_t* total) {
    const uint64_t seq = c->lg_seq;
    const size_t k = seq % LG_SLOTS;
    for (int r = 0; r < c->nranks; ++r) {   // every sender ready before anything is enqueued
        if (r == root) continue;
        khp_ctx* sc = (*c->lgroup)[r];
        if (!sc) return fail(KHP_ENOTREADY, "local group: rank " + std::to_string(r) + " was destroyed");
        if (sc->lg_stamp[k] != seq + 1 || sc->lg_taken[k])
            return fail(KHP_ENOTREADY, "local group: rank " + std::to_string(r) + " has not enqueued gather " +
                                           std::to_string(seq) + " yet");
        if (sc->lg_count[k] != c->gather_counts[r])
            return fail(KHP_EINVAL, "local group: rank " + std::to_string(r) + " packed " +
                                        std::to_string(sc->lg_count[k]) + " pixels, the root's plan expects " +
                                        std::to_string(c->gather_counts[r]) + " (different frame geometry?)");
    }
    *total = 0;
    for (int r = 0; r < c->nranks; ++r) {
        if (r == root) continue;
        khp_ctx* sc = (*c->lgroup)[r];
        HIPCHK(hipStreamWaitEvent(c->stream, sc->lg_evts[k], 0));
        const size_t n = c->gather_counts[r];
        if (n)
            HIPCHK(hipMemcpyAsync(c->stage.as<float>() + *total * 3, sc->lg_slots[k].p, n * 3 * sizeof(float),
                                  hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipEventRecord(sc->lg_copied[k], c->stream));
        sc->lg_taken[k] = true;
        *total += n;
    }
    c->lg_seq = seq + 1;
    return KHP_OK;
}

// RCCL transport: one ncclSend per sender; the root posts one receive per sender
// in ONE group.  The group is closed on every path, also when a receive fails.
// A rank that owns no pixel posts no send, and the root no receive from it
// (both sides know the count from the same plan).
static khp_status rccl_send(khp_ctx* c, uint32_t P, int root) {
    if (P == 0) return KHP_OK;
    hipLaunchKernelGGL(k_pack, dim3((P + 255) / 256), dim3(256), 0, c->stream, c->fb.as<float>(),
                       c->stage_pix.as<uint32_t>(), P, c->stage.as<float>());
    HIPCHK(hipGetLastError());
    HIPCHK(comm_op_begin(c));
    KHPCHK(comm_settle(c, ncclSend(c->stage.p, (size_t)P * 3, ncclFloat32, root, c->comm, c->stream),
                       "ncclSend of " + std::to_string(P) + " pixels to root " + std::to_string(root)));
    HIPCHK(comm_op_end(c));
    return KHP_OK;
}

static khp_status rccl_receive(khp_ctx* c, int root, size_t* total) {
    *total = 0;
    HIPCHK(comm_op_begin(c));
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) return comm_settle(c, r, "ncclGroupStart");
    std::string failed;
    for (int q = 0; q < c->nranks && failed.empty(); ++q) {
        if (q == root || c->gather_counts[q] == 0) continue;
        r = ncclRecv(c->stage.as<float>() + *total * 3, c->gather_counts[q] * 3, ncclFloat32, q, c->comm, c->stream);
        if (r != ncclSuccess && r != ncclInProgress)
            failed = "ncclRecv from rank " + std::to_string(q) + ": " + ncclGetErrorString(r);
        *total += c->gather_counts[q];
    }
    const ncclResult_t e = ncclGroupEnd();   // closes the group on every path
    if (!failed.empty()) {
        (void)comm_settle(c, e, "ncclGroupEnd");
        return comm_abort(c, comm_who(c) + ": " + failed + "; communicator aborted");
    }
    KHPCHK(comm_settle(c, e, "the gather's ncclGroupEnd (receives from every sender)"));
    HIPCHK(comm_op_end(c));
    return KHP_OK;
}

static khp_status gather_now(khp_ctx* c, const khp_render_params* p, int root) {
    khp_status s = check_params(c, p);
    if (s != KHP_OK) return s;
    if (!c->comm && !c->lgroup)
        return fail(KHP_ENOTREADY, c->comm_dead.empty() ? std::string("khp_comm_init first")
                                                        : "the communicator was aborted (" + c->comm_dead +
                                                              "); khp_comm_init again");
    if (!c->fb.p || c->fbW != p->width || c->fbH != p->height) return fail(KHP_ENOTREADY, "render first");
    if (root < 0 || root >= c->nranks) return fail(KHP_EINVAL, "bad root");
    if (p->tile_nranks != (uint32_t)c->nranks) return fail(KHP_EINVAL, "tile_nranks must equal the comm size");
    HIPCHK(hipSetDevice(c->device));
    uint32_t T = p->tile_size ? p->tile_size : 64;
    uint32_t key[6] = {p->width, p->height, T, (uint32_t)c->nranks, (uint32_t)c->rank, (uint32_t)root};
    if (memcmp(key, c->gather_key, sizeof(key)) != 0) {
        // the pixel lists depend only on the frame geometry: build + upload once, not per frame
        std::vector<uint32_t> flat;
        const std::string e = gather_plan(p->width, p->height, T, c->nranks, c->rank, root, c->gather_counts, flat);
        if (!e.empty()) return fail(KHP_EINVAL, "khp_gather_framebuffer: " + e);
        HIPCHK(upload(c->stage_pix, flat.data(), flat.size(), c->stream));
        HIPCHK(c->stage.ensure(flat.size() * 3 * sizeof(float) + 16));
        KHPCHK(wait_stream(c, c->stream, "the gather plan upload"));
        memcpy(c->gather_key, key, sizeof(key));
    }
    // Enqueued on the context stream, which already carries the last frame's
    // join, and not waited for: the next frame's accumulate waits for this
    // gather through fb_evt, and any synchronous call completes it.
    if (!c->gather_evt) HIPCHK(hipEventCreateWithFlags(&c->gather_evt, hipEventDisableTiming));
    if (c->fb_evt) HIPCHK(hipStreamWaitEvent(c->stream, c->fb_evt, 0));
    if (c->rank != root) {
        const uint32_t P = (uint32_t)c->gather_counts[c->rank];
        KHPCHK(c->lgroup ? local_send(c, P) : rccl_send(c, P, root));
    } else {
        // root: receive every other rank's pixels, then scatter them into the framebuffer
        size_t total = 0;
        KHPCHK(c->lgroup ? local_receive(c, root, &total) : rccl_receive(c, root, &total));
        if (total)
            hipLaunchKernelGGL(k_unpack, dim3((uint32_t)((total + 255) / 256)), dim3(256), 0, c->stream,
                               c->fb.as<float>(), c->stage_pix.as<uint32_t>(), (uint32_t)total, c->stage.as<float>());
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(c->gather_evt, c->stream));
    c->fb_evt = c->gather_evt;
    return KHP_OK;
}

#ifdef KHP_LEAF_REUSE
// Diagnostic builds: the leaf-record reuse histograms of the instrumented k_extend
// launches since the last call (traverse.h leaf_reuse), 16 bounces x 8; read and reset.
extern "C" khp_status khp_debug_leaf_reuse(khp_ctx* c, unsigned long long* out) {
    if (!c || !out) return fail(KHP_EINVAL, "null argument");
    KHPCHK(drain(c));
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_leaf_hist), 16 * 8 * sizeof(unsigned long long)));
    static const unsigned long long zero[16 * 8] = {};
    HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_leaf_hist), zero, sizeof(zero)));
    return KHP_OK;
}
#endif

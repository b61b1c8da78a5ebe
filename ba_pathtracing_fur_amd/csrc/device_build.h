// device_build.h -- device-side acceleration-structure build (bvh_build.hip),
// shared by render.hip.  hipcc only.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "scene.h"

namespace khp {

// One owned device allocation (grows, never shrinks).
struct DevMem {
    void* p = nullptr;
    size_t bytes = 0;
    DevMem() = default;
    DevMem(const DevMem&) = delete;
    DevMem& operator=(const DevMem&) = delete;
    ~DevMem() {
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
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const { return (T*)p; }
};

// The BVH as the device build leaves it in HBM.
struct DeviceTree {
    DevMem nodes;  // BuildNode[n_nodes], DFS preorder (the host builder's layout)
    DevMem ids;    // uint32[n_obj], leaf-ordered object ids
    DevMem P;      // uint32[n_obj + 1], leaves starting before each position
    uint32_t n_nodes = 0, n_leaves = 0;
    void release() {
        nodes.release();
        ids.release();
        P.release();
        n_nodes = n_leaves = 0;
    }
};

struct DeviceLayout {
    uint32_t n_dnodes = 0, n_slots = 0;
    int32_t root_ref = 0, root_cnt = 0;
    float root_box[6] = {0, 0, 0, 0, 0, 0};
};

// BVH::addBaseDataStructure on the device from hs.centroid / hs.bounds: the
// host builder's tree (build_bvh), node for node.  Sets hs.depth / hs.max_leaf.
std::string device_build_bvh(HostScene& hs, hipStream_t st, DeviceTree& t, double* kernel_ms);

// make_device_layout on the device: interior records in pair order, leaf slots,
// and the slot-ordered primitive records gathered from hs.rec / hs.aux.
std::string device_layout(const HostScene& hs, DeviceTree& t, hipStream_t st, DevMem& dnodes, DevMem& prims,
                          DevMem& aux, DeviceLayout& out, double* kernel_ms);

// Copy the device tree into hs.nodes / hs.ids (introspection).
std::string download_tree(const DeviceTree& t, HostScene& hs, hipStream_t st);

}  // namespace khp

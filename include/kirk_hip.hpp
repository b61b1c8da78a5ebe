// kirk_hip.hpp -- header-only C++17 convenience layer over the C-ABI in kirk_hip.h.
//
// This is what a C++ host (KIRK's adapter in INTEGRATION.md, or
// examples/render_hairball.cpp) uses.  It adds RAII and exceptions on the host
// side only; everything crossing into libkirk_hip.so is still the plain C ABI.
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "kirk_hip.h"

namespace khp {

struct Error : std::runtime_error {
    khp_status status;
    Error(khp_status s, const std::string& where)
        : std::runtime_error(where + ": " + (khp_last_error() ? khp_last_error() : "")), status(s) {}
};

inline void check(khp_status s, const char* where) {
    if (s != KHP_OK) throw Error(s, where);
}

// Owns the arrays a khp_scene points at (what CPU::Scene::flattenNode would
// hand to the Triangle / Cylinder / Light constructors, CPU_Scene.cpp:73-197).
class SceneBuilder {
  public:
    uint32_t add_material(const khp_material& m) {
        mats_.push_back(m);
        return (uint32_t)mats_.size() - 1;
    }
    // v, n: [count][3][3] world-space vertices / vertex normals (Triangle ctor args)
    void add_triangles(const float* v, const float* n, size_t count, uint32_t mat) {
        tri_v_.insert(tri_v_.end(), v, v + 9 * count);
        tri_n_.insert(tri_n_.end(), n, n + 9 * count);
        tri_mat_.insert(tri_mat_.end(), count, mat);
    }
    // base_r0 / apex_r1: [count][4] (Cylinder ctor args, after the fur flatten adjustments)
    void add_cones(const float* base_r0, const float* apex_r1, size_t count, uint32_t mat) {
        cone_b_.insert(cone_b_.end(), base_r0, base_r0 + 4 * count);
        cone_a_.insert(cone_a_.end(), apex_r1, apex_r1 + 4 * count);
        cone_mat_.insert(cone_mat_.end(), count, mat);
    }
    // fur fibers [n_fibers][verts][3] + radii [n_fibers][verts] -> cones (CPU_Scene.cpp:121-144)
    void add_fibers(const float* positions, const float* radii, uint32_t n_fibers, uint32_t verts, uint32_t mat) {
        size_t nc = (size_t)n_fibers * (verts - 1);
        std::vector<float> b(4 * nc), a(4 * nc);
        check(khp_fibers_to_cones(n_fibers, verts, positions, radii, b.data(), a.data()), "khp_fibers_to_cones");
        add_cones(b.data(), a.data(), nc, mat);
    }
    void add_light(const khp_light& l) { lights_.push_back(l); }
    void set_environment(const khp_environment& e) { env_ = e; }
    void set_camera(const khp_camera& c) { cam_ = c; }
    size_t n_objects() const { return tri_mat_.size() + cone_mat_.size(); }

    // View valid while this builder is alive and unmodified.
    khp_scene view() const {
        khp_scene s{};
        s.n_tris = (uint32_t)tri_mat_.size();
        s.tri_v = tri_v_.data();
        s.tri_n = tri_n_.data();
        s.tri_mat = tri_mat_.data();
        s.n_cones = (uint32_t)cone_mat_.size();
        s.cone_base_r0 = cone_b_.data();
        s.cone_apex_r1 = cone_a_.data();
        s.cone_mat = cone_mat_.data();
        s.n_materials = (uint32_t)mats_.size();
        s.materials = mats_.data();
        s.n_lights = (uint32_t)lights_.size();
        s.lights = lights_.data();
        s.env = env_;
        s.camera = cam_;
        return s;
    }

  private:
    std::vector<float> tri_v_, tri_n_, cone_b_, cone_a_;
    std::vector<uint32_t> tri_mat_, cone_mat_;
    std::vector<khp_material> mats_;
    std::vector<khp_light> lights_;
    khp_environment env_{};
    khp_camera cam_{};
};

// One khp_ctx = one GPU, one HIP stream.  Not copyable; single-threaded like
// KIRK's non-re-entrant PathTracer::render.
class Context {
  public:
    explicit Context(int device = 0, uint32_t flags = 0) { check(khp_create(&c_, device, flags), "khp_create"); }
    ~Context() { khp_destroy(c_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;

    void set_scene(const SceneBuilder& s) {
        khp_scene v = s.view();
        check(khp_set_scene(c_, &v), "khp_set_scene");
    }
    void build_accel() { check(khp_build_accel(c_), "khp_build_accel"); }
    void render(const khp_render_params& p, float* out_rgb = nullptr) {
        check(khp_render(c_, &p, out_rgb), "khp_render");
    }
    // KHP_RENDER_ASYNC renders are complete (and accumulated in call order) after sync()
    void sync() { check(khp_sync(c_), "khp_sync"); }
    void read_framebuffer(float* out_rgb) { check(khp_read_framebuffer(c_, out_rgb), "khp_read_framebuffer"); }
    // 8-bit texture (W*H*4); tm == nullptr: no tonemapping
    void read_rgba8(uint8_t* out_rgba, const khp_tonemap* tm = nullptr) {
        check(khp_read_rgba8(c_, tm, out_rgba), "khp_read_rgba8");
    }
    void trace_closest(uint32_t n, const float* o, const float* d, float* t, int32_t* obj, float* uv = nullptr) {
        check(khp_trace_closest(c_, n, o, d, t, obj, uv), "khp_trace_closest");
    }
    void trace_any(uint32_t n, const float* o, const float* d, const float* tmax, uint8_t* hit) {
        check(khp_trace_any(c_, n, o, d, tmax, hit), "khp_trace_any");
    }
    khp_stats stats() {
        khp_stats s{};
        check(khp_get_stats(c_, &s), "khp_get_stats");
        return s;
    }
    khp_ctx* get() { return c_; }

  private:
    khp_ctx* c_ = nullptr;
};

inline khp_material material(int bsdf, int shader, const float diffuse[3], float ior = 1.52f) {
    khp_material m{};
    m.bsdf = bsdf;
    m.shader = shader;
    for (int i = 0; i < 3; ++i) {
        m.diffuse[i] = diffuse[i];
        m.specular[i] = m.volume[i] = 1.0f;  // Material.h:69-83 defaults
        m.emission[i] = 0.0f;
    }
    m.ior = ior;
    m.roughness = 1.0f;
    return m;
}

}  // namespace khp

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
    // v, n: [count][3][3] world-space vertices / vertex normals (Triangle ctor args);
    // uv: optional [count][3][2] texcoords tca, tcb, tcc (zeros when null)
    void add_triangles(const float* v, const float* n, size_t count, uint32_t mat, const float* uv = nullptr) {
        tri_uv_.resize(6 * tri_mat_.size(), 0.0f);
        tri_v_.insert(tri_v_.end(), v, v + 9 * count);
        tri_n_.insert(tri_n_.end(), n, n + 9 * count);
        tri_mat_.insert(tri_mat_.end(), count, mat);
        if (uv) tri_uv_.insert(tri_uv_.end(), uv, uv + 6 * count);
        else tri_uv_.resize(6 * tri_mat_.size(), 0.0f);
    }
    // A node transform (glm::mat4, column-major) for cones; returns its index.
    uint32_t add_cone_model(const float m[16]) {
        models_.insert(models_.end(), m, m + 16);
        return (uint32_t)(models_.size() / 16 - 1);
    }
    // base_r0 / apex_r1: [count][4] (Cylinder ctor args, after the fur flatten
    // adjustments); model: add_cone_model index (the points are then in the
    // node's object space, as KIRK passes them, CPU_Scene.cpp:136-137) or -1.
    void add_cones(const float* base_r0, const float* apex_r1, size_t count, uint32_t mat, int32_t model = -1) {
        if (model >= 0 && cone_model_.size() < cone_mat_.size()) {  // earlier world-space cones: identity
            const float I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
            cone_model_.resize(cone_mat_.size(), add_cone_model(I));
        }
        cone_b_.insert(cone_b_.end(), base_r0, base_r0 + 4 * count);
        cone_a_.insert(cone_a_.end(), apex_r1, apex_r1 + 4 * count);
        cone_mat_.insert(cone_mat_.end(), count, mat);
        if (model >= 0 || !cone_model_.empty()) {
            uint32_t m = (uint32_t)model;
            if (model < 0) {
                const float I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
                m = add_cone_model(I);
            }
            cone_model_.resize(cone_mat_.size(), m);
        }
    }
    // KIRK::Texture texels (copied): width * height * channels bytes, row y first at y * width * channels
    uint32_t add_texture(const uint8_t* data, uint32_t width, uint32_t height, uint32_t channels,
                         uint32_t wrap_mode = KHP_TEX_WRAP_TILE) {
        texels_.emplace_back(data, data + (size_t)width * height * channels);
        tex_.push_back(khp_texture{width, height, channels, wrap_mode, nullptr});
        return (uint32_t)tex_.size() - 1;
    }
    // texture indices of material mat's parameters (-1: the material value)
    void set_material_textures(uint32_t mat, const khp_material_textures& t) {
        khp_material_textures none{-1, -1, -1, -1, -1};
        if (mtex_.size() <= mat) mtex_.resize(mat + 1, none);
        mtex_[mat] = t;
    }
    void set_environment_map(const khp_env_map& m) { env_map_ = m; }
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
        s.n_cone_models = (uint32_t)(models_.size() / 16);
        s.cone_models = models_.empty() ? nullptr : models_.data();
        s.cone_model = cone_model_.empty() ? nullptr : cone_model_.data();
        tex_view_ = tex_;
        for (size_t i = 0; i < tex_view_.size(); ++i) tex_view_[i].data = texels_[i].data();
        s.n_textures = (uint32_t)tex_view_.size();
        s.textures = tex_view_.empty() ? nullptr : tex_view_.data();
        if (!mtex_.empty()) {
            mtex_view_ = mtex_;
            mtex_view_.resize(mats_.size(), khp_material_textures{-1, -1, -1, -1, -1});
            s.material_textures = mtex_view_.data();
        }
        s.tri_uv = tex_.empty() ? nullptr : tri_uv_.data();
        s.env_map = env_map_;
        return s;
    }

  private:
    std::vector<float> tri_v_, tri_n_, cone_b_, cone_a_, tri_uv_, models_;
    std::vector<uint32_t> tri_mat_, cone_mat_, cone_model_;
    std::vector<std::vector<uint8_t>> texels_;
    std::vector<khp_texture> tex_;
    std::vector<khp_material_textures> mtex_;
    khp_env_map env_map_{};
    mutable std::vector<khp_texture> tex_view_;
    mutable std::vector<khp_material_textures> mtex_view_;
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
    // ABI 13: a moved camera for the next render, nothing rebuilt
    void set_camera(const khp_camera& cam) { check(khp_set_camera(c_, &cam), "khp_set_camera"); }
    // scheduling parameters (ABI 6); never change results
    khp_ctx_params params() {
        khp_ctx_params p{};
        check(khp_get_params(c_, &p), "khp_get_params");
        return p;
    }
    void set_params(const khp_ctx_params& p) { check(khp_set_params(c_, &p), "khp_set_params"); }
    // ABI 7: the light-path variant (KIRK's GLSL lbb_construction / pt_shade bidirectional mode)
    khp_bdpt_params bdpt() {
        khp_bdpt_params p{};
        check(khp_get_bdpt(c_, &p), "khp_get_bdpt");
        return p;
    }
    void set_bdpt(const khp_bdpt_params& p) { check(khp_set_bdpt(c_, &p), "khp_set_bdpt"); }
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

// scene.cpp -- host side of the core: flatten (Triangle / Cylinder ctor
// state), binned-SAH BVH build, device record layout, and the host helpers of
// the C-ABI (camera, fibers -> cones, seeded generators, registries).
// Built with -ffp-contract=off so every float matches the device and the
// documented semantics bit-for-bit.
#include "scene.h"
#include "objects.h"

#include <string.h>

#include <algorithm>
#include <cfloat>
#include <thread>

namespace khp {



// Light ctors + QuadLight::calcParams + Light::transform(identity)
// (Common/Light.h ctors, Light.cpp:112-118, 216-220, 263-276).
void light_init(DevLight& L, const khp_light& in) {
    memset(&L, 0, sizeof(L));
    L.kind = in.kind;
    for (int i = 0; i < 3; ++i) {
        L.color[i] = in.color[i];
        L.position[i] = in.position[i];
    }
    L.c = in.att_const;
    L.l = in.att_lin;
    L.q = in.att_quad;
    L.radius = in.radius;
    v3 dir1 = normalize(ld3(in.direction));
    if (in.kind == KHP_LIGHT_POINT) dir1 = normalize(mk(0.0f, 0.0f, 0.0f));
    if (in.kind == KHP_LIGHT_SPOT) {
        L.outer = in.outer_angle;
        L.inner = (in.inner_angle < 0.0f || in.inner_angle > in.outer_angle) ? in.outer_angle : in.inner_angle;
    }
    if (in.kind == KHP_LIGHT_QUAD) {
        v3 n = dir1, s;
        if (fabsf(n.x) > fabsf(n.y)) s = mk(-n.z, 0.0f, n.x) / sqrtf(n.x * n.x + n.z * n.z);
        else s = mk(0.0f, n.z, -n.y) / sqrtf(n.y * n.y + n.z * n.z);
        v3 t = cross(n, s);
        float sx = in.size[0], sy = in.size[1];
        v3 p = ld3(in.position);
        v3 vs[4] = {(p + (s * -sx) / 2.0f) + (t * -sy) / 2.0f, (p + (s * sx) / 2.0f) + (t * -sy) / 2.0f,
                    (p + (s * sx) / 2.0f) + (t * sy) / 2.0f, (p + (s * -sx) / 2.0f) + (t * sy) / 2.0f};
        for (int k = 0; k < 4; ++k) {
            L.vert[k][0] = vs[k].x;
            L.vert[k][1] = vs[k].y;
            L.vert[k][2] = vs[k].z;
        }
        L.radius = sqrtf((sx * sy) / PIF);
    }
    v3 d = normalize(dir1);
    L.direction[0] = d.x;
    L.direction[1] = d.y;
    L.direction[2] = d.z;
}

// Triangle::Triangle / Cylinder::Cylinder (objects.h, shared with the device flatten).
static void tri_ctor(HostScene& hs, uint32_t id, v3 a, v3 b, v3 c, v3 na, v3 nb, v3 nc, uint32_t mat,
                     const float* uv) {
    tri_object(a, b, c, na, nb, nc, &hs.rec[16 * (size_t)id], &hs.bounds[6 * (size_t)id],
               &hs.centroid[3 * (size_t)id], &hs.tri_nrm[9 * (size_t)id], uv,
               hs.tri_uv.empty() ? nullptr : &hs.tri_uv[6 * (size_t)id]);
    hs.aux[id] = Aux{0.0f, mat, id, 0u};  // flags: triangle
}

static void cone_ctor(HostScene& hs, uint32_t id, uint32_t ci, v3 base, v3 apex, float r0, float r1, uint32_t mat,
                      int model) {
    float* rec = &hs.rec[16 * (size_t)id];
    float* bnd = &hs.bounds[6 * (size_t)id];
    float* cen = &hs.centroid[3 * (size_t)id];
    const float base_d = model < 0 ? cone_object(base, apex, r0, r1, rec, bnd, cen)
                                   : cone_object_xf(base, apex, r0, r1, &hs.models[25 * (size_t)model],
                                                    &hs.models[25 * (size_t)model + 16], rec, bnd, cen);
    if (!hs.cone_h.empty()) hs.cone_h[ci] = length(apex - base);  // Cylinder::m_height (pre-transform)
    hs.aux[id] = Aux{base_d, mat, id, 1u};  // flags: cone
}

std::string scene_models(const khp_scene* s, HostScene& hs) {
    hs.models.clear();
    if (s->n_cone_models == 0) {
        if (s->cone_model) return "cone_model given without cone_models";
        return std::string();
    }
    if (!s->cone_models) return "cone_models missing";
    hs.models.resize(25 * (size_t)s->n_cone_models);
    for (uint32_t k = 0; k < s->n_cone_models; ++k) {
        float* o = &hs.models[25 * (size_t)k];
        memcpy(o, s->cone_models + 16 * (size_t)k, 16 * sizeof(float));
        mat4_inverse_transpose3(o, o + 16);
    }
    return std::string();
}

std::string scene_textures(const khp_scene* s, HostScene& hs) {
    hs.tex.clear();
    hs.texels.clear();
    hs.mtex.clear();
    hs.env_map = s->env_map;
    hs.textured = false;
    if (s->n_textures && !s->textures) return "textures missing";
    size_t off = 0;
    for (uint32_t i = 0; i < s->n_textures; ++i) {
        const khp_texture& t = s->textures[i];
        if (t.width == 0 || t.height == 0 || !t.data) return "texture without texels";
        if (t.channels < 1 || t.channels > 4) return "texture channels must be 1..4";
        if ((uint64_t)t.width * t.height >= (1ull << 31)) return "texture too large";
        hs.tex.push_back(DevTexture{t.width, t.height, t.channels, t.wrap_mode, (uint64_t)off});
        off += (size_t)t.width * t.height * t.channels;
    }
    hs.texels.resize(off);
    for (uint32_t i = 0; i < s->n_textures; ++i) {
        const khp_texture& t = s->textures[i];
        memcpy(hs.texels.data() + hs.tex[i].off, t.data, (size_t)t.width * t.height * t.channels);
    }
    auto valid = [&](int32_t k) { return k >= -1 && k < (int32_t)s->n_textures; };
    hs.mtex.assign(s->n_materials, DevMatTex{{-1, -1, -1, -1, -1}});
    if (s->material_textures) {
        for (uint32_t m = 0; m < s->n_materials; ++m) {
            const khp_material_textures& mt = s->material_textures[m];
            const int32_t k[5] = {mt.diffuse, mt.specular, mt.volume, mt.emission, mt.roughness};
            for (int j = 0; j < 5; ++j) {
                if (!valid(k[j])) return "material texture index out of range";
                hs.mtex[m].t[j] = k[j];
                hs.textured = hs.textured || k[j] >= 0;
            }
        }
    }
    const khp_env_map& e = s->env_map;
    if (e.type < KHP_ENV_COLOR || e.type > KHP_ENV_SPHERE_MAP) return "unknown environment type";
    const int nmaps = e.type == KHP_ENV_CUBE_MAP ? 6 : e.type == KHP_ENV_SPHERE_MAP ? 1 : 0;
    for (int j = 0; j < nmaps; ++j)
        if (e.tex[j] < 0 || e.tex[j] >= (int32_t)s->n_textures) return "environment map texture index out of range";
    hs.textured = hs.textured || nmaps > 0;
    return std::string();
}

std::string flatten_scene(const khp_scene* s, HostScene& hs, bool objects) {
    if (!s) return "scene is null";
    uint64_t n = (uint64_t)s->n_tris + s->n_cones;
    if (n == 0) return "Your scene is empty!";  // BoundingBox.cpp:121-122
    if (n >= (1ull << 31)) return "too many objects";
    if (s->n_tris && (!s->tri_v || !s->tri_n || !s->tri_mat)) return "triangle arrays missing";
    if (s->n_cones && (!s->cone_base_r0 || !s->cone_apex_r1 || !s->cone_mat)) return "cone arrays missing";
    if (s->n_materials == 0 || !s->materials) return "no materials";
    if (s->n_lights && !s->lights) return "lights missing";
    for (uint32_t i = 0; i < s->n_materials; ++i) {
        const khp_material& m = s->materials[i];
        if (m.bsdf < 0 || m.bsdf >= KHP_BSDF_COUNT) return "unknown BSDF kind";
        if (m.shader < 0 || m.shader >= KHP_SHADER_COUNT) return "unknown shader kind";
    }
    for (uint32_t i = 0; i < s->n_lights; ++i)
        if (s->lights[i].kind < 0 || s->lights[i].kind > KHP_LIGHT_SUN) return "unknown light kind";
    hs = HostScene();
    hs.n_tris = s->n_tris;
    hs.n_cones = s->n_cones;
    hs.n_obj = (uint32_t)n;
    std::string err = scene_textures(s, hs);
    if (!err.empty()) return err;
    err = scene_models(s, hs);
    if (!err.empty()) return err;
    if (!objects) {  // the device flattens the objects (flatten.hip)
        hs.mats.assign(s->materials, s->materials + s->n_materials);
        hs.lights.resize(s->n_lights);
        for (uint32_t i = 0; i < s->n_lights; ++i) light_init(hs.lights[i], s->lights[i]);
        hs.env = s->env;
        hs.cam = s->camera;
        return std::string();
    }
    hs.rec.resize(16 * n);
    hs.aux.resize(n);
    hs.bounds.resize(6 * n);
    hs.centroid.resize(3 * n);
    hs.tri_nrm.resize(9 * (size_t)s->n_tris);
    if (s->tri_frame) hs.tri_frame.assign(s->tri_frame, s->tri_frame + 9 * (size_t)s->n_tris);
    else hs.tri_frame.assign(9 * (size_t)s->n_tris, 0.0f);
    for (uint32_t i = 0; i < s->n_tris; ++i)
        if (s->tri_mat[i] >= s->n_materials) return "triangle material index out of range";
    for (uint32_t i = 0; i < s->n_cones; ++i)
        if (s->cone_mat[i] >= s->n_materials) return "cone material index out of range";
    if (s->cone_model)
        for (uint32_t i = 0; i < s->n_cones; ++i)
            if (s->cone_model[i] >= s->n_cone_models) return "cone model index out of range";
    if (hs.textured) {
        hs.tri_uv.assign(6 * (size_t)s->n_tris, 0.0f);
        hs.cone_h.assign(s->n_cones, 0.0f);
    }
    unsigned nt = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
    auto work = [&](unsigned t) {
        for (uint32_t i = t; i < s->n_tris; i += nt) {
            const float* v = s->tri_v + 9 * (size_t)i;
            const float* nn = s->tri_n + 9 * (size_t)i;
            tri_ctor(hs, i, ld3(v), ld3(v + 3), ld3(v + 6), ld3(nn), ld3(nn + 3), ld3(nn + 6), s->tri_mat[i],
                     s->tri_uv ? s->tri_uv + 6 * (size_t)i : nullptr);
        }
        for (uint32_t i = t; i < s->n_cones; i += nt) {
            const float* b = s->cone_base_r0 + 4 * (size_t)i;
            const float* a = s->cone_apex_r1 + 4 * (size_t)i;
            const int model = s->n_cone_models == 0 ? -1 : s->cone_model ? (int)s->cone_model[i] : 0;
            cone_ctor(hs, s->n_tris + i, i, ld3(b), ld3(a), b[3], a[3], s->cone_mat[i], model);
        }
    };
    if (n < 65536) nt = 1;
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& t : th) t.join();
    hs.mats.assign(s->materials, s->materials + s->n_materials);
    hs.lights.resize(s->n_lights);
    for (uint32_t i = 0; i < s->n_lights; ++i) light_init(hs.lights[i], s->lights[i]);
    hs.env = s->env;
    hs.cam = s->camera;
    return std::string();
}

// ---- binned SAH BVH (CPU_BVH.cpp:16-44, 95-138, 357-552; BoundingBox.cpp) ----
struct Box {
    v3 mn, mx;
};
static inline float smin(float a, float b) { return (b < a) ? b : a; }  // std::min
static inline float smax(float a, float b) { return (a < b) ? b : a; }  // std::max
static inline Box box_empty() { return Box{mk(FLT_MAX, FLT_MAX, FLT_MAX), mk(-FLT_MAX, -FLT_MAX, -FLT_MAX)}; }
static inline void grow(Box& b, v3 p) {
    b.mn = mk(smin(b.mn.x, p.x), smin(b.mn.y, p.y), smin(b.mn.z, p.z));
    b.mx = mk(smax(b.mx.x, p.x), smax(b.mx.y, p.y), smax(b.mx.z, p.z));
}
static inline void grow(Box& b, const Box& o) {
    b.mn = mk(smin(b.mn.x, o.mn.x), smin(b.mn.y, o.mn.y), smin(b.mn.z, o.mn.z));
    b.mx = mk(smax(b.mx.x, o.mx.x), smax(b.mx.y, o.mx.y), smax(b.mx.z, o.mx.z));
}
static inline float area(const Box& b) {
    v3 s = b.mx - b.mn;
    return 2.0f * (s.x * s.y + s.x * s.z + s.y * s.z);
}
static inline bool worth(const Box& b) {
    v3 d = b.mx - b.mn;
    return d.x > 0.0f && d.y > 0.0f && d.z > 0.0f;
}

struct Builder {
    HostScene& hs;
    const float* cen;
    uint32_t* ids;
    float cget(uint32_t oid, int axis) const { return cen[3 * (size_t)oid + axis]; }
    v3 cvec(uint32_t oid) const { return ld3(&cen[3 * (size_t)oid]); }

    void partition(uint32_t first, uint32_t second, uint32_t& lsec, uint32_t& rfirst, const Box& cb, Box& lcb,
                   Box& rcb) const {
        float best = FLT_MAX;
        int best_axis = 0, best_plane = 0;
        constexpr int NB = 16, NP = 15;
        float cbmins[3], ks[3];
        for (int axis = 0; axis < 3; ++axis) {
            const float cbmin = comp(cb.mn, axis);
            const float cbmax = comp(cb.mx, axis);
            const float cbdiff = cbmax - cbmin;
            const float epsilon = 0.1f;
            const float k = ((float)NB * (1.0f - epsilon)) / cbdiff;
            cbmins[axis] = cbmin;
            ks[axis] = k;
            Box bb[NB];
            uint32_t bn[NB];
            for (int i = 0; i < NB; ++i) { bb[i] = box_empty(); bn[i] = 0; }
            for (uint32_t id = first; id <= second; ++id) {
                uint32_t oid = ids[id];
                int bin = (int)(k * (cget(oid, axis) - cbmin));
                grow(bb[bin], cvec(oid));
                ++bn[bin];
            }
            uint32_t ln[NP];
            Box lb[NP];
            lb[0] = box_empty();
            grow(lb[0], bb[0]);
            ln[0] = bn[0];
            for (int p = 1; p < NP; ++p) {
                lb[p] = box_empty();
                grow(lb[p], lb[p - 1]);
                grow(lb[p], bb[p]);
                ln[p] = ln[p - 1] + bn[p];
            }
            uint32_t rn[NP];
            Box rb[NP];
            for (int p = NP - 1; p >= 0; --p) {
                rb[p] = box_empty();
                grow(rb[p], bb[p + 1]);
                rn[p] = bn[p + 1];
                if (p != NP - 1) {
                    grow(rb[p], rb[p + 1]);
                    rn[p] += rn[p + 1];
                }
                float cost = area(lb[p]) * (float)ln[p] + area(rb[p]) * (float)rn[p];
                if (cost < best) {
                    best = cost;
                    best_axis = axis;
                    best_plane = p;
                    lcb = lb[p];
                    rcb = rb[p];
                }
            }
        }
        const float cbmin = cbmins[best_axis], k = ks[best_axis];
        int left = (int)first, right = (int)second;
        bool ls = false, rs = false;
        while (left < right) {
            if (!ls) {
                int b = (int)(k * (cget(ids[left], best_axis) - cbmin));
                if (b > best_plane) ls = true;
                else ++left;
            }
            if (!rs) {
                int b = (int)(k * (cget(ids[right], best_axis) - cbmin));
                if (b <= best_plane) rs = true;
                else --right;
            }
            if (ls && rs) {
                std::swap(ids[left], ids[right]);
                ls = rs = false;
                ++left;
                --right;
            }
        }
        if (left > right) { lsec = (uint32_t)right; rfirst = (uint32_t)left; }
        else if (ls) { lsec = (uint32_t)(left - 1); rfirst = (uint32_t)left; }
        else if (rs) { lsec = (uint32_t)right; rfirst = (uint32_t)(right + 1); }
        else {
            int b = (int)(k * (cget(ids[left], best_axis) - cbmin));
            if (b > best_plane) { lsec = (uint32_t)(left - 1); rfirst = (uint32_t)left; }
            else { lsec = (uint32_t)left; rfirst = (uint32_t)(left + 1); }
        }
    }

    // BVHNode::split; nodes appended to `out` in DFS preorder, child indices relative to `out`.
    int32_t split(uint32_t first, uint32_t second, const Box& cb, uint32_t depth, std::vector<BuildNode>& out,
                  uint32_t& maxdepth, uint32_t& maxleaf, int par) const {
        int32_t ni = (int32_t)out.size();
        out.push_back(BuildNode{});
        Box bv = box_empty();
        const float* bounds = hs.bounds.data();
        for (uint32_t id = first; id <= second; ++id) {
            const float* b = &bounds[6 * (size_t)ids[id]];
            bv.mn = mk(smin(bv.mn.x, b[0]), smin(bv.mn.y, b[1]), smin(bv.mn.z, b[2]));
            bv.mx = mk(smax(bv.mx.x, b[3]), smax(bv.mx.y, b[4]), smax(bv.mx.z, b[5]));
        }
        out[ni].mn = bv.mn;
        out[ni].mx = bv.mx;
        if (depth > maxdepth) maxdepth = depth;
        if (second - first > 1u && worth(cb)) {
            uint32_t lsec, rfirst;
            Box lcb, rcb;
            partition(first, second, lsec, rfirst, cb, lcb, rcb);
            out[ni].count = 0;
            if (par > 0 && second - first > 32768u) {
                std::vector<BuildNode> L, R;
                uint32_t ld = 0, rd = 0, lm = 0, rm = 0;
                std::thread t([&] { split(first, lsec, lcb, depth + 1, L, ld, lm, par - 1); });
                split(rfirst, second, rcb, depth + 1, R, rd, rm, par - 1);
                t.join();
                int32_t lbase = (int32_t)out.size();
                for (auto nd : L) {
                    if (nd.count == 0) { nd.left += lbase; nd.right += lbase; }
                    out.push_back(nd);
                }
                int32_t rbase = (int32_t)out.size();
                for (auto nd : R) {
                    if (nd.count == 0) { nd.left += rbase; nd.right += rbase; }
                    out.push_back(nd);
                }
                out[ni].left = lbase;
                out[ni].right = rbase;
                maxdepth = std::max(maxdepth, std::max(ld, rd));
                maxleaf = std::max(maxleaf, std::max(lm, rm));
            } else {
                int32_t l = split(first, lsec, lcb, depth + 1, out, maxdepth, maxleaf, 0);
                int32_t r = split(rfirst, second, rcb, depth + 1, out, maxdepth, maxleaf, 0);
                out[ni].left = l;
                out[ni].right = r;
            }
        } else {
            out[ni].first = (int32_t)first;
            out[ni].count = (int32_t)(second - first + 1);
            out[ni].left = out[ni].right = -1;
            maxleaf = std::max(maxleaf, second - first + 1);
        }
        return ni;
    }
};

void build_bvh(HostScene& hs, int n_threads) {
    hs.ids.resize(hs.n_obj);
    Box cb = box_empty();
    for (uint32_t i = 0; i < hs.n_obj; ++i) {
        hs.ids[i] = i;
        grow(cb, ld3(&hs.centroid[3 * (size_t)i]));
    }
    Builder b{hs, hs.centroid.data(), hs.ids.data()};
    hs.nodes.clear();
    hs.nodes.reserve(2 * (size_t)hs.n_obj);
    int par = 0;
    while ((1 << par) < n_threads && par < 8) ++par;
    hs.depth = 0;
    hs.max_leaf = 0;
    b.split(0, hs.n_obj - 1, cb, 1, hs.nodes, hs.depth, hs.max_leaf, par);
}

void make_device_layout(HostScene& hs) {
    // Interior records: the two children of a node, when both are interior, get
    // the records (2k, 2k+1) of one 128-B line, so the traversal can expand a
    // far sibling from the line it fetched for the near one.  A lone interior
    // child takes a whole pair (even index).  The root sits alone in pair 0.
    const size_t nn = hs.nodes.size();
    std::vector<int32_t> rec_of(nn, -1);
    int32_t next = 0;
    if (hs.nodes[0].count == 0) {
        rec_of[0] = 0;
        next = 2;
        std::vector<int32_t> st{0};
        while (!st.empty()) {
            int32_t i = st.back();
            st.pop_back();
            const BuildNode& n = hs.nodes[i];
            const bool li = hs.nodes[n.left].count == 0, ri = hs.nodes[n.right].count == 0;
            if (li) rec_of[n.left] = next;
            if (ri) rec_of[n.right] = li ? next + 1 : next;
            if (li || ri) next += 2;
            if (ri) st.push_back(n.right);
            if (li) st.push_back(n.left);  // left subtree first: DFS preorder of pairs
        }
    }
    hs.dnodes.assign((size_t)next, DevNode{});
    // Leaf slots: a leaf with >= 2 candidates starts at an even slot so its
    // first two 64-B records share one line (pad slots are never referenced).
    std::vector<uint32_t> slot_of_first(hs.n_obj + 1, 0);
    uint32_t ns = 0;
    for (size_t i = 0; i < nn; ++i) {  // preorder visits leaves in ids order
        const BuildNode& n = hs.nodes[i];
        if (n.count == 0) continue;
        if (n.count >= 2 && (ns & 1u)) ++ns;
        slot_of_first[n.first] = ns;
        ns += (uint32_t)n.count;
    }
    hs.n_slots = ns;
    auto child_ref = [&](int32_t c, int32_t& ref, int32_t& cnt) {
        const BuildNode& n = hs.nodes[c];
        if (n.count > 0) {
            uint32_t ce = (uint32_t)n.count < LEAF_CNT_ESC ? (uint32_t)n.count : LEAF_CNT_ESC;
            ref = (int32_t)(LEAF_BIT | (ce << 24) | slot_of_first[n.first]);
            cnt = n.count;
        } else {
            ref = rec_of[c];
            cnt = 0;
        }
    };
    for (size_t i = 0; i < nn; ++i) {
        const BuildNode& n = hs.nodes[i];
        if (n.count != 0) continue;
        DevNode& d = hs.dnodes[rec_of[i]];
        const BuildNode& L = hs.nodes[n.left];
        const BuildNode& R = hs.nodes[n.right];
        float a[4] = {L.mn.x, L.mn.y, L.mn.z, L.mx.x};
        float b[4] = {L.mx.y, L.mx.z, R.mn.x, R.mn.y};
        float c[4] = {R.mn.z, R.mx.x, R.mx.y, R.mx.z};
        memcpy(d.a, a, sizeof(a));
        memcpy(d.b, b, sizeof(b));
        memcpy(d.c, c, sizeof(c));
        child_ref(n.left, d.ref[0], d.cnt[0]);
        child_ref(n.right, d.ref[1], d.cnt[1]);
    }
    child_ref(0, hs.root_ref, hs.root_cnt);
    const BuildNode& r = hs.nodes[0];
    float rb[6] = {r.mn.x, r.mn.y, r.mn.z, r.mx.x, r.mx.y, r.mx.z};
    memcpy(hs.root_box, rb, sizeof(rb));
    hs.slot_rec.assign(16 * (size_t)ns, 0.0f);
    hs.slot_aux.assign(ns, Aux{0.0f, 0u, 0u, 0u});
    for (size_t i = 0; i < nn; ++i) {
        const BuildNode& n = hs.nodes[i];
        if (n.count == 0) continue;
        const uint32_t s0 = slot_of_first[n.first];
        for (int32_t k = 0; k < n.count; ++k) {
            const uint32_t o = hs.ids[(size_t)n.first + k], sl = s0 + (uint32_t)k;
            memcpy(&hs.slot_rec[16 * (size_t)sl], &hs.rec[16 * (size_t)o], 16 * sizeof(float));
            hs.slot_aux[sl] = hs.aux[o];
        }
        hs.slot_aux[s0].flags |= (uint32_t)n.count << 8;
    }
}

// Tile t (row-major over the frame) belongs to rank t % nranks;
// KIRK's own segmentation is square segments in order (BufferSegmentation.h:34-75).
void owned_pixels(uint32_t W, uint32_t H, uint32_t T, uint32_t rank, uint32_t nranks, std::vector<uint32_t>& out) {
    out.clear();
    const uint32_t tx_n = (W + T - 1) / T, ty_n = (H + T - 1) / T;
    const uint32_t bpr = T / 8;
    for (uint32_t tid = 0; tid < tx_n * ty_n; ++tid) {
        if (nranks > 1 && tid % nranks != rank) continue;
        const uint32_t tx = tid % tx_n, ty = tid / tx_n;
        for (uint32_t blk = 0; blk < bpr * bpr; ++blk) {
            const uint32_t bx = blk % bpr, by = blk / bpr;
            for (uint32_t j = 0; j < 64; ++j) {
                const uint32_t x = tx * T + bx * 8 + (j & 7), y = ty * T + by * 8 + (j >> 3);
                if (x < W && y < H) out.push_back(y * W + x);
            }
        }
    }
}

// Root: every other rank's owned pixels, in rank order (what it receives).
// Sender: its own owned pixels (what it sends).  Both sides therefore agree on
// counts[sender] for every sender, which is what ncclSend/ncclRecv need.
std::string gather_plan(uint32_t W, uint32_t H, uint32_t T, int nranks, int rank, int root,
                        std::vector<uint64_t>& counts, std::vector<uint32_t>& flat) {
    if (W == 0 || H == 0) return "empty frame";
    if (T == 0 || T % 8 != 0) return "tile size must be a positive multiple of 8";
    if (nranks < 1 || rank < 0 || rank >= nranks || root < 0 || root >= nranks) return "bad rank/root";
    counts.assign((size_t)nranks, 0);
    flat.clear();
    std::vector<uint32_t> one;
    for (int r = 0; r < nranks; ++r) {
        if (r == root) continue;               // the root's own tiles stay in place
        if (rank != root && r != rank) continue;  // a sender lists only itself
        owned_pixels(W, H, T, (uint32_t)r, (uint32_t)nranks, one);
        counts[(size_t)r] = one.size();
        flat.insert(flat.end(), one.begin(), one.end());
    }
    return std::string();
}

}  // namespace khp

// ============================================================================
//  C-ABI host helpers
// ============================================================================
using namespace khp;

static thread_local std::string g_err;
khp_status khp::fail(khp_status s, const std::string& msg) {
    g_err = msg;
    return s;
}
const char* khp::last_error() { return g_err.c_str(); }

extern "C" khp_status khp_host_build(const khp_scene* scene, uint32_t* n_nodes, uint32_t* depth, float* node_boxes,
                                     int32_t* node_first, int32_t* node_count, int32_t* object_ids,
                                     float* obj_bounds, float* records) {
    if (!scene || !n_nodes) return fail(KHP_EINVAL, "scene or n_nodes is null");
    HostScene hs;
    std::string err = flatten_scene(scene, hs);
    if (!err.empty()) return fail(KHP_EINVAL, err);
    unsigned nt = std::max(1u, std::min(32u, std::thread::hardware_concurrency()));
    build_bvh(hs, (int)nt);
    *n_nodes = (uint32_t)hs.nodes.size();
    if (depth) *depth = hs.depth;
    for (size_t i = 0; i < hs.nodes.size(); ++i) {
        const BuildNode& n = hs.nodes[i];
        if (node_boxes) {
            float b[6] = {n.mn.x, n.mn.y, n.mn.z, n.mx.x, n.mx.y, n.mx.z};
            memcpy(node_boxes + 6 * i, b, sizeof(b));
        }
        if (node_first) node_first[i] = n.count ? n.first : -1;
        if (node_count) node_count[i] = n.count;
    }
    for (uint32_t i = 0; i < hs.n_obj; ++i) {
        if (object_ids) object_ids[i] = (int32_t)hs.ids[i];
        if (obj_bounds) {
            memcpy(obj_bounds + 9 * (size_t)i, &hs.bounds[6 * (size_t)i], 6 * sizeof(float));
            memcpy(obj_bounds + 9 * (size_t)i + 6, &hs.centroid[3 * (size_t)i], 3 * sizeof(float));
        }
        if (records) memcpy(records + 16 * (size_t)i, &hs.rec[16 * (size_t)i], 16 * sizeof(float));
    }
    return KHP_OK;
}

extern "C" khp_status khp_gather_plan(uint32_t width, uint32_t height, uint32_t tile_size, int nranks, int rank,
                                      int root, uint64_t* counts, uint32_t* pixels, uint64_t* n_pixels) {
    if (!n_pixels) return fail(KHP_EINVAL, "khp_gather_plan: n_pixels is null");
    std::vector<uint64_t> cnt;
    std::vector<uint32_t> flat;
    const std::string e = gather_plan(width, height, tile_size ? tile_size : 64, nranks, rank, root, cnt, flat);
    if (!e.empty()) return fail(KHP_EINVAL, "khp_gather_plan: " + e);
    *n_pixels = flat.size();
    if (counts) memcpy(counts, cnt.data(), cnt.size() * sizeof(uint64_t));
    if (pixels) memcpy(pixels, flat.data(), flat.size() * sizeof(uint32_t));
    return KHP_OK;
}

static const char* kBsdfNames[KHP_BSDF_COUNT] = {
    "LambertianReflectionBSDF", "SpecularReflectionBSDF", "SpecularTransmissionBSDF", "GlossyBSDF",
    "GlassBSDF", "MilkGlassBSDF", "LambertianTransmissionBSDF", "EmissionBSDF", "TransparentBSDF",
    "MarschnerHairBSDF", "DEonHairBSDF"};

extern "C" int khp_bsdf_kind_from_name(const char* name) {
    if (!name) return -1;
    for (int i = 0; i < KHP_BSDF_COUNT; ++i)
        if (strcmp(name, kBsdfNames[i]) == 0) return i;
    return -1;
}
extern "C" const char* khp_bsdf_name(int kind) {
    return (kind >= 0 && kind < KHP_BSDF_COUNT) ? kBsdfNames[kind] : nullptr;
}
extern "C" int khp_shader_kind_from_name(const char* name) {
    if (!name) return -1;
    // ShaderFactory names (SimpleShader.h:29, MarschnerHairShader.h:29)
    if (strcmp(name, "SimpleShader") == 0) return KHP_SHADER_SIMPLE;
    if (strcmp(name, "MarschnerHairShader") == 0) return KHP_SHADER_MARSCHNER_HAIR;
    return -1;
}

// Camera::applyParameters (Common/Camera.cpp:6-37), identity node transform.
extern "C" khp_status khp_camera_setup(const float position[3], const float look_at[3], const float up[3],
                                       float sensor_w, float sensor_h, float focal_length, uint32_t width,
                                       uint32_t height, khp_camera* out) {
    if (!position || !look_at || !up || !out || width == 0 || height == 0 || focal_length <= 0.0f)
        return fail(KHP_EINVAL, "camera: null pointer, zero resolution or focal length <= 0");
    v3 pos = ld3(position), la = ld3(look_at), upv = ld3(up);
    // KIRK would produce a NaN frame here (normalize of a zero vector); reject it instead
    v3 side = cross(upv, la);
    if (dot(la, la) == 0.0f || dot(side, side) == 0.0f)
        return fail(KHP_EINVAL, "degenerate camera frame (look direction zero or parallel to up)");
    float aspect = (float)width / (float)height;
    v3 az = normalize(-la);
    v3 ax = normalize(cross(upv, az));
    v3 ay = normalize(cross(az, ax));
    float diam = sqrtf(sensor_w * sensor_w + sensor_h * sensor_h);
    float fov = 2.0f * k_atanf(diam / (2.0f * focal_length));
    float half = 0.5f * fov;
    float sy = k_sinf(half) / k_cosf(half);
    float sx = sy * aspect;
    float px = 2.0f * sx / (float)width;
    v3 bl = ((pos - az) - ay * sy) - ax * sx;
    for (int i = 0; i < 3; ++i) {
        out->position[i] = comp(pos, i);
        out->bottom_left[i] = comp(bl, i);
        out->axis_x[i] = comp(ax, i);
        out->axis_y[i] = comp(ay, i);
    }
    out->pixel_size = px;
    return KHP_OK;
}

// CPU_Scene::flattenNode fiber -> Cylinder arguments (CPU_Scene.cpp:121-144).
extern "C" khp_status khp_fibers_to_cones(uint32_t n_fibers, uint32_t verts, const float* positions,
                                          const float* radii, float* out_base_r0, float* out_apex_r1) {
    if (verts < 2 || !positions || !radii || !out_base_r0 || !out_apex_r1) return KHP_EINVAL;
    size_t k = 0;
    for (uint32_t f = 0; f < n_fibers; ++f) {
        const float* P = positions + (size_t)f * verts * 3;
        const float* R = radii + (size_t)f * verts;
        for (uint32_t c = 0; c + 1 < verts; ++c, ++k) fiber_segment(P, R, c, out_base_r0 + 4 * k, out_apex_r1 + 4 * k);
    }
    return KHP_OK;
}

extern "C" khp_status khp_fibers_to_triangles(uint32_t n_fibers, uint32_t verts, const float* positions,
                                              const float* radii, uint32_t res, float* out_v, float* out_n,
                                              float* out_frame) {
    if (verts < 2 || res == 0 || !positions || !radii || !out_v || !out_n || !out_frame) return KHP_EINVAL;
    const uint32_t per_seg = 2 * res * res;
    size_t k = 0;
    for (uint32_t f = 0; f < n_fibers; ++f) {
        const float* P = positions + (size_t)f * verts * 3;
        const float* R = radii + (size_t)f * verts;
        for (uint32_t c = 0; c + 1 < verts; ++c)
            for (uint32_t t = 0; t < per_seg; ++t, ++k)
                fiber_tube_triangle(P, R, c, res, t, out_v + 9 * k, out_n + 9 * k, out_frame + 9 * k);
    }
    return KHP_OK;
}

// Seeded hairball: Mesh::addFurToFaces recurrence (Mesh.cpp:118-142) in each
// root's tangent frame (local y = sphere normal, local z = random tangent).
extern "C" khp_status khp_gen_hairball(uint32_t n, uint32_t verts, const float center[3], float ball_r,
                                       float root_r, uint32_t seed, float* positions, float* radii) {
    if (verts < 2 || verts > 64 || !center || !positions || !radii) return KHP_EINVAL;
    // glm::log((float)i) for i = 0..64 (float-rounded natural logs)
    static float lnt[65];
    static bool init = false;
    if (!init) {
        for (int i = 1; i <= 64; ++i) lnt[i] = (float)log((double)i);
        init = true;
    }
    const v3 C = ld3(center);
    const uint32_t key0 = lowbias32(seed ^ 0x48414952u);
    for (uint32_t s = 0; s < n; ++s)
        hairball_strand(s, verts, C, ball_r, root_r, key0, lnt, positions + (size_t)s * verts * 3,
                        radii + (size_t)s * verts);
    return KHP_OK;
}

static void push_tri(std::vector<float>& v, std::vector<float>& n, v3 a, v3 b, v3 c, v3 na, v3 nb, v3 nc) {
    v3 vs[3] = {a, b, c}, ns[3] = {na, nb, nc};
    for (int i = 0; i < 3; ++i) {
        v.push_back(vs[i].x); v.push_back(vs[i].y); v.push_back(vs[i].z);
        n.push_back(ns[i].x); n.push_back(ns[i].y); n.push_back(ns[i].z);
    }
}

extern "C" khp_status khp_gen_icosphere(uint32_t subdiv, const float center[3], float radius, float* tri_v,
                                        float* tri_n) {
    if (subdiv > 8 || !center || !tri_v || !tri_n) return KHP_EINVAL;
    const float t = 1.61803398874989484820f;
    std::vector<v3> P = {mk(-1, t, 0), mk(1, t, 0), mk(-1, -t, 0), mk(1, -t, 0), mk(0, -1, t), mk(0, 1, t),
                         mk(0, -1, -t), mk(0, 1, -t), mk(t, 0, -1), mk(t, 0, 1), mk(-t, 0, -1), mk(-t, 0, 1)};
    for (auto& p : P) p = normalize(p);
    std::vector<uint32_t> F = {0, 11, 5, 0, 5, 1, 0, 1, 7, 0, 7, 10, 0, 10, 11, 1, 5, 9, 5, 11, 4, 11, 10, 2,
                               10, 7, 6, 7, 1, 8, 3, 9, 4, 3, 4, 2, 3, 2, 6, 3, 6, 8, 3, 8, 9, 4, 9, 5, 2, 4, 11,
                               6, 2, 10, 8, 6, 7, 9, 8, 1};
    for (uint32_t s = 0; s < subdiv; ++s) {
        std::vector<uint32_t> G;
        G.reserve(F.size() * 4);
        for (size_t i = 0; i < F.size(); i += 3) {
            uint32_t a = F[i], b = F[i + 1], c = F[i + 2];
            v3 ab = normalize((P[a] + P[b]) * 0.5f), bc = normalize((P[b] + P[c]) * 0.5f),
               ca = normalize((P[c] + P[a]) * 0.5f);
            uint32_t iab = (uint32_t)P.size(); P.push_back(ab);
            uint32_t ibc = (uint32_t)P.size(); P.push_back(bc);
            uint32_t ica = (uint32_t)P.size(); P.push_back(ca);
            uint32_t q[12] = {a, iab, ica, b, ibc, iab, c, ica, ibc, iab, ibc, ica};
            G.insert(G.end(), q, q + 12);
        }
        F.swap(G);
    }
    v3 C = ld3(center);
    std::vector<float> vv, nn;
    for (size_t i = 0; i < F.size(); i += 3) {
        v3 a = P[F[i]], b = P[F[i + 1]], c = P[F[i + 2]];
        push_tri(vv, nn, C + a * radius, C + b * radius, C + c * radius, a, b, c);
    }
    memcpy(tri_v, vv.data(), vv.size() * sizeof(float));
    memcpy(tri_n, nn.data(), nn.size() * sizeof(float));
    return KHP_OK;
}

extern "C" khp_status khp_gen_torus(uint32_t nu, uint32_t nv, const float center[3], float R, float r,
                                    float* tri_v, float* tri_n) {
    if (nu < 3 || nv < 3 || !center || !tri_v || !tri_n) return KHP_EINVAL;
    v3 C = ld3(center);
    auto P = [&](uint32_t i, uint32_t j, v3& pos, v3& nrm) {
        float a = 2.0f * PIF * (float)(i % nu) / (float)nu;
        float b = 2.0f * PIF * (float)(j % nv) / (float)nv;
        float ca = k_cosf(a), sa = k_sinf(a), cb = k_cosf(b), sb = k_sinf(b);
        nrm = mk(ca * cb, sb, sa * cb);
        pos = C + mk((R + r * cb) * ca, r * sb, (R + r * cb) * sa);
    };
    size_t k = 0;
    for (uint32_t i = 0; i < nu; ++i)
        for (uint32_t j = 0; j < nv; ++j) {
            v3 p00, n00, p10, n10, p01, n01, p11, n11;
            P(i, j, p00, n00); P(i + 1, j, p10, n10); P(i, j + 1, p01, n01); P(i + 1, j + 1, p11, n11);
            v3 tv[6] = {p00, p01, p10, p10, p01, p11}, tn[6] = {n00, n01, n10, n10, n01, n11};
            for (int q = 0; q < 6; ++q, ++k) {
                tri_v[3 * k] = tv[q].x; tri_v[3 * k + 1] = tv[q].y; tri_v[3 * k + 2] = tv[q].z;
                tri_n[3 * k] = tn[q].x; tri_n[3 * k + 1] = tn[q].y; tri_n[3 * k + 2] = tn[q].z;
            }
        }
    return KHP_OK;
}

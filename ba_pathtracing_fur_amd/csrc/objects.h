// objects.h -- per-object scene preparation shared by the host flatten
// (scene.cpp, g++) and the device flatten (flatten.hip, hipcc): one source, so
// both produce the same bits (both built with -ffp-contract=off).
//   Triangle::Triangle            Common/Triangle.cpp:3-129 (identity model matrix)
//   Cylinder::Cylinder/computeBounds  Common/Cylinder.cpp:5-67, 306-336
//   CPU_Scene::flattenNode fibers CPU_Scene.cpp:121-144
//   Mesh::addFurToFaces recurrence Mesh.cpp:111-142 (seeded hairball stand-in)
#pragma once

#include <cfloat>

#include "kmath.h"

namespace khp {

constexpr float OBJ_RAY_EPS = 1e-4f;          // KIRK::cRayEpsilon (Common/Ray.h:9)
constexpr uint32_t OBJ_TRI_TAG = 0x7fc0deadu;  // == TRI_TAG (scene.h)

KHD void obj_set_comp(v3& a, int i, float v) {
    if (i == 0) a.x = v;
    else if (i == 1) a.y = v;
    else a.z = v;
}

// Triangle ctor: vertices reordered by the longest AABB axis, edges with the
// zero-guard, smooth normals normalized.  rec: (A, tag) (ab, 0) (ac, 0) (0);
// bounds: bmin.xyz bmax.xyz; cen: centroid; nrm: nA nB nC; uv_out (optional):
// the texcoords tca tcb tcc of uv_in (6 floats, or zeros when null) in the
// same order (Triangle.cpp:31-110 permutes m_tca/m_tcb/m_tcc with the vertices).
KHD void tri_object(v3 a, v3 b, v3 c, v3 na, v3 nb, v3 nc, float* rec, float* bounds, float* cen, float* nrm,
                    const float* uv_in = nullptr, float* uv_out = nullptr) {
    v3 bmin = vmin(vmin(a, b), c) - mk(OBJ_RAY_EPS, OBJ_RAY_EPS, OBJ_RAY_EPS);
    v3 bmax = vmax(vmax(a, b), c) + mk(OBJ_RAY_EPS, OBJ_RAY_EPS, OBJ_RAY_EPS);
    v3 diff = bmax - bmin;
    int lA = 0;
    float longest = diff.x;
    if (diff.y > longest) { longest = diff.y; lA = 1; }
    if (diff.z > longest) { longest = diff.z; lA = 2; }
    v3 Na = normalize(na), Nb = normalize(nb), Nc = normalize(nc);
    v3 A = a, B = b, C = c, nA = Na, nB = Nb, nC = Nc;
    float ca = comp(a, lA), cb = comp(b, lA), cc = comp(c, lA);
    // six orderings, later matches override earlier ones (ties); o* = source vertex of A, B, C
    int oA = 0, oB = 1, oC = 2;
    if (ca <= cb && cb <= cc) { A = a; B = b; C = c; nA = Na; nB = Nb; nC = Nc; oA = 0; oB = 1; oC = 2; }
    if (cb <= ca && ca <= cc) { A = b; B = a; C = c; nA = Nb; nB = Na; nC = Nc; oA = 1; oB = 0; oC = 2; }
    if (ca <= cc && cc <= cb) { A = a; B = c; C = b; nA = Na; nB = Nc; nC = Nb; oA = 0; oB = 2; oC = 1; }
    if (cc <= ca && ca <= cb) { A = c; B = a; C = b; nA = Nc; nB = Na; nC = Nb; oA = 2; oB = 0; oC = 1; }
    if (cb <= cc && cc <= ca) { A = b; B = c; C = a; nA = Nb; nB = Nc; nC = Na; oA = 1; oB = 2; oC = 0; }
    if (cc <= cb && cb <= ca) { A = c; B = b; C = a; nA = Nc; nB = Nb; nC = Na; oA = 2; oB = 1; oC = 0; }
    if (uv_out) {
        const int o[3] = {oA, oB, oC};
        for (int k = 0; k < 3; ++k) {
            uv_out[2 * k] = uv_in ? uv_in[2 * o[k]] : 0.0f;
            uv_out[2 * k + 1] = uv_in ? uv_in[2 * o[k] + 1] : 0.0f;
        }
    }
    v3 ab = B - A, ac = C - A, bc = C - B;
    if (comp(ab, lA) == 0.0f) obj_set_comp(ab, lA, 0.0001f);
    if (comp(ac, lA) == 0.0f) obj_set_comp(ac, lA, 0.0001f);
    if (comp(bc, lA) == 0.0f) obj_set_comp(bc, lA, 0.0001f);
    v3 ce = ((A + B) + C) / 3.0f;
    rec[0] = A.x; rec[1] = A.y; rec[2] = A.z; rec[3] = f_from_bits(OBJ_TRI_TAG);
    rec[4] = ab.x; rec[5] = ab.y; rec[6] = ab.z; rec[7] = 0.0f;
    rec[8] = ac.x; rec[9] = ac.y; rec[10] = ac.z; rec[11] = 0.0f;
    rec[12] = 0.0f; rec[13] = 0.0f; rec[14] = 0.0f; rec[15] = 0.0f;
    bounds[0] = bmin.x; bounds[1] = bmin.y; bounds[2] = bmin.z;
    bounds[3] = bmax.x; bounds[4] = bmax.y; bounds[5] = bmax.z;
    cen[0] = ce.x; cen[1] = ce.y; cen[2] = ce.z;
    nrm[0] = nA.x; nrm[1] = nA.y; nrm[2] = nA.z;
    nrm[3] = nB.x; nrm[4] = nB.y; nrm[5] = nB.z;
    nrm[6] = nC.x; nrm[7] = nC.y; nrm[8] = nC.z;
}

// Cylinder ctor: frame (u, v, w), slope, axial extent, AABB of the rotated
// local box, centroid at 40 % of the axis.  rec: (base, r0) (u, slope)
// (v, min_d) (w, max_d); returns base_d = dot(base, v).
KHD float cone_object(v3 base, v3 apex, float r0, float r1, float* rec, float* bounds, float* cen) {
    v3 v = apex - base;
    float height = length(v);
    v = normalize(v);
    v3 tmp = mk(0.0f, 1.0f, 0.0f);
    if (1.0f - fabsf(dot(tmp, v)) < OBJ_RAY_EPS) tmp = mk(0.0f, 0.0f, 1.0f);
    v3 u = normalize(cross(v, tmp));
    v3 w = normalize(cross(u, v));
    u = normalize(u);
    v = normalize(v);
    w = normalize(w);
    float slope = (r0 - r1) / height;
    float base_d = dot(base, v);
    float min_d = dot(v, base), max_d = dot(v, apex);
    if (max_d < min_d) {
        float t = min_d;
        min_d = max_d;
        max_d = t;
    }
    float radius = (r0 > r1) ? r0 + 1e-6f : r1 + 1e-6f;
    v3 l0 = mk(-radius, 0.0f, -radius), l1 = mk(radius, height, radius);
    v3 corners[8] = {mk(l0.x, l1.y, l1.z), mk(l0.x, l0.y, l1.z), mk(l1.x, l0.y, l1.z), mk(l1.x, l1.y, l1.z),
                     mk(l1.x, l1.y, l0.z), mk(l1.x, l0.y, l0.z), mk(l0.x, l0.y, l0.z), mk(l0.x, l1.y, l0.z)};
    v3 bmin = mk(FLT_MAX, FLT_MAX, FLT_MAX), bmax = mk(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (int i = 0; i < 8; ++i) {
        v3 q = corners[i];
        v3 P = mk((u.x * q.x + v.x * q.y) + w.x * q.z, (u.y * q.x + v.y * q.y) + w.y * q.z,
                  (u.z * q.x + v.z * q.y) + w.z * q.z) + base;
        if (P.x < bmin.x) bmin.x = P.x;
        if (P.x > bmax.x) bmax.x = P.x;
        if (P.y < bmin.y) bmin.y = P.y;
        if (P.y > bmax.y) bmax.y = P.y;
        if (P.z < bmin.z) bmin.z = P.z;
        if (P.z > bmax.z) bmax.z = P.z;
    }
    v3 ce = base + (apex - base) * 0.4f;  // Cylinder.cpp:50
    rec[0] = base.x; rec[1] = base.y; rec[2] = base.z; rec[3] = r0;
    rec[4] = u.x; rec[5] = u.y; rec[6] = u.z; rec[7] = slope;
    rec[8] = v.x; rec[9] = v.y; rec[10] = v.z; rec[11] = min_d;
    rec[12] = w.x; rec[13] = w.y; rec[14] = w.z; rec[15] = max_d;
    bounds[0] = bmin.x; bounds[1] = bmin.y; bounds[2] = bmin.z;
    bounds[3] = bmax.x; bounds[4] = bmax.y; bounds[5] = bmax.z;
    cen[0] = ce.x; cen[1] = ce.y; cen[2] = ce.z;
    return base_d;
}

// ---- glm 0.9.9 matrix arithmetic, in its operation order (column-major:
// M[4*c + r] = m[c][r]) ----------------------------------------------------------
// vec3(M * vec4(p, w)): ((m0 x + m1 y) + (m2 z + m3 w))  (type_mat4x4.inl operator*)
KHD v3 mat4_apply(const float* M, v3 p, float w) {
    float o[3];
    for (int r = 0; r < 3; ++r) o[r] = (M[r] * p.x + M[4 + r] * p.y) + (M[8 + r] * p.z + M[12 + r] * w);
    return mk(o[0], o[1], o[2]);
}

// mat3 * vec3: (m[0][r] x + m[1][r] y) + m[2][r] z  (type_mat3x3.inl operator*)
KHD v3 mat3_apply(const float* A, v3 v) {
    float o[3];
    for (int r = 0; r < 3; ++r) o[r] = (A[r] * v.x + A[3 + r] * v.y) + A[6 + r] * v.z;
    return mk(o[0], o[1], o[2]);
}

// glm::mat3(glm::transpose(glm::inverse(M))) (func_matrix.inl compute_inverse<4,4>:
// cofactor pairs, SignA/SignB, determinant from the first row and column).
// out: 3x3 column-major.
KHD void mat4_inverse_transpose3(const float* M, float* out) {
#define m(c, r) M[4 * (c) + (r)]
    const float c00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3), c02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3);
    const float c03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3), c04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3);
    const float c06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3), c07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
    const float c08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2), c10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2);
    const float c11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2), c12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3);
    const float c14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3), c15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
    const float c16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2), c18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2);
    const float c19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2), c20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1);
    const float c22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1), c23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);
    const float fac[6][4] = {{c00, c00, c02, c03}, {c04, c04, c06, c07}, {c08, c08, c10, c11},
                             {c12, c12, c14, c15}, {c16, c16, c18, c19}, {c20, c20, c22, c23}};
    const float vec[4][4] = {{m(1, 0), m(0, 0), m(0, 0), m(0, 0)}, {m(1, 1), m(0, 1), m(0, 1), m(0, 1)},
                             {m(1, 2), m(0, 2), m(0, 2), m(0, 2)}, {m(1, 3), m(0, 3), m(0, 3), m(0, 3)}};
    // Inv_k = Vec_a * Fac_b - Vec_c * Fac_d + Vec_e * Fac_f, column k of the inverse (times its sign)
    const int ia[4][6] = {{1, 0, 2, 1, 3, 2}, {0, 0, 2, 3, 3, 4}, {0, 1, 1, 3, 3, 5}, {0, 2, 1, 4, 2, 5}};
    float inv[4][4];
    for (int k = 0; k < 4; ++k) {
        const float sgn0 = (k & 1) ? -1.0f : 1.0f;  // SignA (+,-,+,-) for k even, SignB for k odd
        for (int i = 0; i < 4; ++i) {
            const float x = (vec[ia[k][0]][i] * fac[ia[k][1]][i] - vec[ia[k][2]][i] * fac[ia[k][3]][i]) +
                            vec[ia[k][4]][i] * fac[ia[k][5]][i];
            inv[k][i] = x * ((i & 1) ? -sgn0 : sgn0);
        }
    }
    // Dot0 = m[0] * Row0, Row0 = (inv[0][0], inv[1][0], inv[2][0], inv[3][0])
    const float d0 = m(0, 0) * inv[0][0], d1 = m(0, 1) * inv[1][0], d2 = m(0, 2) * inv[2][0], d3 = m(0, 3) * inv[3][0];
    const float one_over_det = 1.0f / ((d0 + d1) + (d2 + d3));
    // transpose, upper-left 3x3: out[c][r] = inverse[r][c]
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) out[3 * c + r] = inv[r][c] * one_over_det;
#undef m
}

// Cylinder ctor with a node transform (Cylinder.cpp:5-67; flattenNode passes
// base_transform * child->m_transform, CPU_Scene.cpp:119,136-137): base/apex
// transformed by M; the frame (u, v, w) and the height come from the
// PRE-transform points and the frame is then mapped by M_ti and renormalised;
// slope uses the pre-transform height; min_d / max_d / base_d use the
// transformed points; the centroid is the transformed base + 0.4 x the
// pre-transform axis (Cylinder.cpp:50).  Mti = mat4_inverse_transpose3(M).
KHD float cone_object_xf(v3 base_in, v3 apex_in, float r0, float r1, const float* M, const float* Mti, float* rec,
                         float* bounds, float* cen) {
    const v3 base = mat4_apply(M, base_in, 1.0f), apex = mat4_apply(M, apex_in, 1.0f);
    v3 v = apex_in - base_in;
    const float height = length(v);
    v = normalize(v);
    v3 tmp = mk(0.0f, 1.0f, 0.0f);
    if (1.0f - fabsf(dot(tmp, v)) < OBJ_RAY_EPS) tmp = mk(0.0f, 0.0f, 1.0f);
    v3 u = normalize(cross(v, tmp));
    v3 w = normalize(cross(u, v));
    u = normalize(mat3_apply(Mti, u));
    v = normalize(mat3_apply(Mti, v));
    w = normalize(mat3_apply(Mti, w));
    const float slope = (r0 - r1) / height;
    const float base_d = dot(base, v);
    float min_d = dot(v, base), max_d = dot(v, apex);
    if (max_d < min_d) {
        const float t = min_d;
        min_d = max_d;
        max_d = t;
    }
    const float radius = (r0 > r1) ? r0 + 1e-6f : r1 + 1e-6f;
    const v3 l0 = mk(-radius, 0.0f, -radius), l1 = mk(radius, height, radius);
    const v3 corners[8] = {mk(l0.x, l1.y, l1.z), mk(l0.x, l0.y, l1.z), mk(l1.x, l0.y, l1.z), mk(l1.x, l1.y, l1.z),
                           mk(l1.x, l1.y, l0.z), mk(l1.x, l0.y, l0.z), mk(l0.x, l0.y, l0.z), mk(l0.x, l1.y, l0.z)};
    v3 bmin = mk(FLT_MAX, FLT_MAX, FLT_MAX), bmax = mk(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (int i = 0; i < 8; ++i) {
        const v3 q = corners[i];
        const v3 P = mk((u.x * q.x + v.x * q.y) + w.x * q.z, (u.y * q.x + v.y * q.y) + w.y * q.z,
                        (u.z * q.x + v.z * q.y) + w.z * q.z) + base;
        if (P.x < bmin.x) bmin.x = P.x;
        if (P.x > bmax.x) bmax.x = P.x;
        if (P.y < bmin.y) bmin.y = P.y;
        if (P.y > bmax.y) bmax.y = P.y;
        if (P.z < bmin.z) bmin.z = P.z;
        if (P.z > bmax.z) bmax.z = P.z;
    }
    const v3 ce = base + (apex_in - base_in) * 0.4f;
    rec[0] = base.x; rec[1] = base.y; rec[2] = base.z; rec[3] = r0;
    rec[4] = u.x; rec[5] = u.y; rec[6] = u.z; rec[7] = slope;
    rec[8] = v.x; rec[9] = v.y; rec[10] = v.z; rec[11] = min_d;
    rec[12] = w.x; rec[13] = w.y; rec[14] = w.z; rec[15] = max_d;
    bounds[0] = bmin.x; bounds[1] = bmin.y; bounds[2] = bmin.z;
    bounds[3] = bmax.x; bounds[4] = bmax.y; bounds[5] = bmax.z;
    cen[0] = ce.x; cen[1] = ce.y; cen[2] = ce.z;
    return base_d;
}

// One fiber segment c (vertices c, c+1) -> cone: base pulled back by 0.8 % of
// the segment, base radius shrunk 5 % (c <= 3) or 10 %.
KHD void fiber_segment(const float* P, const float* R, uint32_t c, float* ob, float* oa) {
    v3 basepos = ld3(P + 3 * c), apexpos = ld3(P + 3 * (c + 1));
    float br = R[c];
    basepos = basepos - (apexpos - basepos) * 0.008f;
    br -= (c > 3) ? 0.1f * br : 0.05f * br;
    ob[0] = basepos.x; ob[1] = basepos.y; ob[2] = basepos.z; ob[3] = br;
    oa[0] = apexpos.x; oa[1] = apexpos.y; oa[2] = apexpos.z; oa[3] = R[c + 1];
}

// glm::mat4(1) * vec4(p, w), in glm's operation order ((m0 x + m1 y) + (m2 z + m3 w)):
// exact, up to the sign of zero components (the identity mesh transform of
// fiberToTriangles; the inverse-transpose for normals is the same matrix).
KHD v3 ident_apply(v3 p, float w) {
    const float x = (1.0f * p.x + 0.0f * p.y) + (0.0f * p.z + 0.0f * w);
    const float y = (0.0f * p.x + 1.0f * p.y) + (0.0f * p.z + 0.0f * w);
    const float z = (0.0f * p.x + 0.0f * p.y) + (1.0f * p.z + 0.0f * w);
    return mk(x, y, z);
}

// fiberToTriangles (CPU_Scene.cpp:232-345) for segment c of one fiber: its
// frame (no base pull-back / radius shrink on this path), then triangle t of
// the 2 res^2 triangles: cells (i, j) row by row, two triangles per cell.
// ov / on / of: 9 floats each (3 vertices, 3 normals, frame u v w).
KHD void fiber_tube_triangle(const float* P, const float* R, uint32_t c, uint32_t res, uint32_t t, float* ov,
                             float* on, float* of) {
    const v3 base = ld3(P + 3 * c), apex = ld3(P + 3 * (c + 1));
    v3 v = apex - base;
    const float height = length(v);
    v = normalize(v);
    v3 tmp = mk(0.0f, 1.0f, 0.0f);
    if (1.0f - fabsf(dot(tmp, v)) < OBJ_RAY_EPS) tmp = mk(0.0f, 0.0f, 1.0f);
    const v3 u = normalize(cross(v, tmp));
    const v3 w = normalize(cross(u, v));
    const float slope = (R[c] - R[c + 1]) / height;
    const uint32_t cell = t >> 1, j = cell / res, i = cell % res;
    // tri1: (i, j+1) (i, j) (i+1, j); tri2: (i+1, j) (i+1, j+1) (i, j+1)
    const uint32_t gi[2][3] = {{i, i, i + 1}, {i + 1, i + 1, i}};
    const uint32_t gj[2][3] = {{j + 1, j, j}, {j, j + 1, j + 1}};
    for (int k = 0; k < 3; ++k) {
        const uint32_t ii = gi[t & 1][k], jj = gj[t & 1][k];
        const float uu = (float)ii / (float)res;
        const float phi = 2.0f * PIF * uu;
        const float vv = height * ((float)jj / (float)res);
        const float radius = R[c] - slope * vv;
        const v3 q = ((base + u * (radius * k_sinf(phi))) + v * vv) + w * (radius * k_cosf(phi));
        const float tt = dot(q, v) - dot(base, v);
        const v3 q1 = q - v * tt;
        v3 n = normalize(q1 - base);
        n = normalize(n + v * slope);
        const v3 qv = ident_apply(q, 1.0f);
        const v3 nv = normalize(ident_apply(n, 0.0f));
        ov[3 * k] = qv.x; ov[3 * k + 1] = qv.y; ov[3 * k + 2] = qv.z;
        on[3 * k] = nv.x; on[3 * k + 1] = nv.y; on[3 * k + 2] = nv.z;
    }
    of[0] = u.x; of[1] = u.y; of[2] = u.z;
    of[3] = v.x; of[4] = v.y; of[5] = v.z;
    of[6] = w.x; of[7] = w.y; of[8] = w.z;
}

// Strand s of the seeded hairball: root uniform on the sphere, the
// addFurToFaces recurrence in the root's tangent frame.  lnt[i] = (float)ln(i).
KHD void hairball_strand(uint32_t s, uint32_t verts, v3 C, float ball_r, float root_r, uint32_t key0,
                         const float* lnt, float* P, float* R) {
    uint32_t key = lowbias32(key0 ^ s);
    float u0 = draw_u01(key, 0), u1 = draw_u01(key, 1), u2 = draw_u01(key, 2);
    float z = 1.0f - 2.0f * u0;
    float rxy = sqrtf(gmax(0.0f, 1.0f - z * z));
    float phi = 2.0f * PIF * u1;
    v3 nrm = mk(rxy * k_cosf(phi), z, rxy * k_sinf(phi));
    v3 ref = fabsf(nrm.y) < 0.9f ? mk(0.0f, 1.0f, 0.0f) : mk(1.0f, 0.0f, 0.0f);
    v3 t0 = normalize(cross(nrm, ref));
    v3 b0 = cross(nrm, t0);
    float psi = 2.0f * PIF * u2;
    v3 tan = t0 * k_cosf(psi) + b0 * k_sinf(psi);
    v3 pos = C + nrm * ball_r;
    pos = pos - nrm * 0.003f;  // "move start position down" (Mesh.cpp:115)
    float radius = root_r;
    P[0] = pos.x; P[1] = pos.y; P[2] = pos.z;
    R[0] = radius;
    uint32_t k = 1;
    for (int i = (int)verts; i > 1; --i, ++k) {
        float off_y = lnt[i] / 90.0f;
        v3 point = (pos + nrm * off_y) + tan * 0.06f;
        radius -= radius / ((float)i + 5.0f);
        P[3 * k] = point.x; P[3 * k + 1] = point.y; P[3 * k + 2] = point.z;
        R[k] = radius;
        pos = point;
    }
    R[verts - 1] = 0.001f;  // Mesh.cpp:142
}

}  // namespace khp

// render_hairball.cpp -- C++ host program on the C-ABI (no Python, no torch).
//
// Builds BASELINE config 3 (seeded hairball on a diffuse plane, 2x2 quad light,
// sky) exactly like ba_pathtracing_fur_amd.scenes.config3, renders it with the
// HIP core and optionally writes the fp32 radiance as a PFM (or, for a .ppm
// name, the tonemapped 8-bit texture from the device output stage).  This is the
// shape of KIRK's host side calling the core and doubles as a
// C++ bench:
//
//   render_hairball [strands=1000000] [W=1920] [H=1080] [spp=8] [depth=5] [frames=3] [out.pfm]
//                   [light_paths=0]
// light_paths > 0 renders with the light-path (bidirectional) variant (ABI 7,
// khp_set_bdpt): that many subpaths per light, 4 vertices, both connection passes.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/kirk_hip.hpp"

static void quad(khp::SceneBuilder& sb, const float p[4][3], const float n[3], uint32_t mat) {
    const int idx[2][3] = {{0, 1, 2}, {0, 2, 3}};
    float v[2][3][3], nn[2][3][3];
    for (int t = 0; t < 2; ++t)
        for (int k = 0; k < 3; ++k)
            for (int c = 0; c < 3; ++c) {
                v[t][k][c] = p[idx[t][k]][c];
                nn[t][k][c] = n[c];
            }
    sb.add_triangles(&v[0][0][0], &nn[0][0][0], 2, mat);
}

int main(int argc, char** argv) {
    const uint32_t strands = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000000u;
    const uint32_t W = argc > 2 ? (uint32_t)atoi(argv[2]) : 1920u, H = argc > 3 ? (uint32_t)atoi(argv[3]) : 1080u;
    const uint32_t spp = argc > 4 ? (uint32_t)atoi(argv[4]) : 8u, depth = argc > 5 ? (uint32_t)atoi(argv[5]) : 5u;
    const int frames = argc > 6 ? atoi(argv[6]) : 3;
    const char* out = argc > 7 && strcmp(argv[7], "-") != 0 ? argv[7] : nullptr;
    const uint32_t light_paths = argc > 8 ? (uint32_t)atoi(argv[8]) : 0u;
    const uint32_t SEED = 0x4B49524Bu;
    try {
        khp::SceneBuilder sb;
        const float grey[3] = {0.5f, 0.5f, 0.5f}, brown[3] = {0.545f, 0.353f, 0.169f};
        uint32_t m_plane = sb.add_material(khp::material(KHP_BSDF_LAMBERTIAN_REFLECTION, KHP_SHADER_SIMPLE, grey));
        const float P[4][3] = {{-6, 0, -6}, {-6, 0, 6}, {6, 0, 6}, {6, 0, -6}}, up[3] = {0, 1, 0};
        quad(sb, P, up, m_plane);
        // hairball (Mesh::addFurToFaces recurrence on sphere roots) -> cones (CPU_Scene.cpp:121-144)
        const uint32_t verts = 10;
        std::vector<float> pos((size_t)strands * verts * 3), rad((size_t)strands * verts);
        const float centre[3] = {0.0f, 1.0f, 0.0f};
        khp::check(khp_gen_hairball(strands, verts, centre, 1.0f, 0.004f, SEED, pos.data(), rad.data()),
                   "khp_gen_hairball");
        uint32_t m_fur = sb.add_material(khp::material(KHP_BSDF_MARSCHNER_HAIR, KHP_SHADER_MARSCHNER_HAIR, brown, 1.55f));
        sb.add_fibers(pos.data(), rad.data(), strands, verts, m_fur);
        khp_light L{};
        L.kind = KHP_LIGHT_QUAD;
        const float lp[3] = {0, 3, 0}, ld[3] = {0, -1, 0};
        for (int i = 0; i < 3; ++i) {
            L.color[i] = 5.0f;
            L.position[i] = lp[i];
            L.direction[i] = ld[i];
        }
        L.size[0] = L.size[1] = 2.0f;
        L.att_const = 1.0f;
        sb.add_light(L);
        khp_environment env{{0.7f, 0.9f, 1.0f}, {0.1f, 0.1f, 0.1f}};
        sb.set_environment(env);
        khp_camera cam{};
        const float cpos[3] = {0.0f, 1.4f, 4.6f}, look[3] = {0.0f, -0.12f, -1.0f};
        khp::check(khp_camera_setup(cpos, look, up, 0.036f, 0.024f, 0.0415f, W, H, &cam), "khp_camera_setup");
        sb.set_camera(cam);

        khp::Context ctx(0);
        if (light_paths > 0) {
            khp_bdpt_params bd;
            khp_bdpt_params_defaults(&bd);
            bd.enabled = 1;
            bd.light_paths = light_paths;
            bd.vertices = 4;
            ctx.set_bdpt(bd);
        }
        auto t0 = std::chrono::steady_clock::now();
        ctx.set_scene(sb);
        ctx.build_accel();
        double build_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        khp_render_params p{W, H, spp, depth, SEED, 0, 64, 0, 1, KHP_RENDER_NO_READBACK};
        ctx.render(p);  // warm-up
        // pipelined frames (ABI 5): enqueue every frame, complete them with one sync;
        // the stats report then sums the frames (divided below)
        khp_render_params pa = p;
        pa.flags |= KHP_RENDER_ASYNC;
        t0 = std::chrono::steady_clock::now();
        for (int f = 0; f < frames; ++f) ctx.render(pa);
        ctx.sync();
        double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        khp_stats st = ctx.stats();
        const double nf = st.frames ? (double)st.frames : 1.0;
        st.extend_ms /= nf;
        st.shade_ms /= nf;
        st.shadow_ms /= nf;
        printf("{\"objects\": %zu, \"build_s\": %.2f, \"frames\": %d, \"ms_per_frame\": %.3f, \"Msamples_per_s\": %.2f, "
               "\"extend_ms\": %.2f, \"shade_ms\": %.2f, \"shadow_ms\": %.2f}\n",
               sb.n_objects(), build_s, frames, dt / frames * 1e3, (double)W * H * spp * frames / dt / 1e6,
               st.extend_ms, st.shade_ms, st.shadow_ms);
        const size_t olen = out ? strlen(out) : 0;
        if (out && olen > 4 && strcmp(out + olen - 4, ".ppm") == 0) {
            // 8-bit texture on the device, after Tonemapper::map with gamma 2.2
            khp_tonemap tm;
            khp_tonemap_defaults(&tm);
            tm.gamma = 2.2f;
            std::vector<uint8_t> rgba((size_t)W * H * 4);
            ctx.read_rgba8(rgba.data(), &tm);
            FILE* f = fopen(out, "wb");
            if (!f) throw std::runtime_error("cannot open output");
            fprintf(f, "P6\n%u %u\n255\n", W, H);
            for (uint32_t y = H; y-- > 0;)  // PPM rows are top-to-bottom; row 0 of the texture is the bottom
                for (uint32_t x = 0; x < W; ++x) fwrite(&rgba[((size_t)y * W + x) * 4], 1, 3, f);
            fclose(f);
        } else if (out) {
            std::vector<float> fb((size_t)W * H * 3);
            ctx.read_framebuffer(fb.data());
            FILE* f = fopen(out, "wb");
            if (!f) throw std::runtime_error("cannot open output");
            fprintf(f, "PF\n%u %u\n-1.0\n", W, H);  // PFM rows are bottom-to-top, like the framebuffer
            fwrite(fb.data(), sizeof(float), fb.size(), f);
            fclose(f);
        }
    } catch (const khp::Error& e) {
        fprintf(stderr, "error (%d): %s\n", (int)e.status, e.what());
        return 1;
    } catch (const std::exception& e) {
        fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}

/*
 * standalone_cornell.cpp — a compiled C++ caller of the drop-in boundary: the
 * reference's headless render loop (Standalone/StandaloneRenderManager.cpp:55-140:
 * initialize, initScene, renderNextIteration(i, i, radius, ...), the PPM radius
 * schedule r^2 <- r^2 (i + alpha) / (i + 1) in double, getOutputBuffer) driving the
 * Cornell scene (scene/Cornell.cpp:20-207) through OptixRenderer.cpp -> liborx.so.
 *
 *   standalone_cornell --method ppm|pt|vcm --width W --height H --photon-launch P
 *                      --iterations N --seed S --out output.f32
 *   standalone_cornell --print-camera W H      (aspect-corrected fov, no device needed)
 *
 * Writes the W*H*3 float running sum (the reference's output buffer) to --out.
 */
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <stdexcept>
#include <vector>

#include "OptixRenderer.h"

/* Cornell.cpp: five Lambert walls, an area light under the ceiling, registered once */
class Cornell : public IScene {
public:
    Cornell() {
        const float lp[3] = {343.0f, 548.7999f, 227.0f}, lv1[3] = {0.0f, 0.0f, 105.0f}, lv2[3] = {-130.0f, 0.0f, 0.0f};
        orx_light L = {};
        L.type = ORX_LIGHT_AREA;
        const float pw[3] = {0.5e6f, 0.4e6f, 0.2e6f};
        for (int k = 0; k < 3; k++) {
            L.power[k] = pw[k];
            L.position[k] = lp[k];
            L.v1[k] = lv1[k];
            L.v2[k] = lv2[k];
        }
        m_lights.push_back(L);
        /* Light.cpp:14-28: inverse area 1/|v1 x v2| in float */
        const float cx = lv1[1] * lv2[2] - lv1[2] * lv2[1], cy = lv1[2] * lv2[0] - lv1[0] * lv2[2],
                    cz = lv1[0] * lv2[1] - lv1[1] * lv2[0];
        const float inv_area = 1.0f / std::sqrt((cx * cx + cy * cy) + cz * cz);
        const uint32_t white = material(ORX_MAT_DIFFUSE, 0.8f, 0.8f, 0.8f);
        const uint32_t green = material(ORX_MAT_DIFFUSE, 0.05f, 0.8f, 0.05f);
        const uint32_t red = material(ORX_MAT_DIFFUSE, 1.0f, 0.05f, 0.05f);
        quad(0, 0, 0, 0, 0, 559.2f, 556.0f, 0, 0, white);         /* floor */
        quad(0, 548.80f, 0, 556.0f, 0, 0, 0, 0, 559.2f, white);   /* ceiling */
        quad(0, 0, 559.2f, 0, 548.8f, 0, 556.0f, 0, 0, white);    /* back wall */
        quad(0, 0, 0, 0, 548.8f, 0, 0, 0, 559.2f, green);         /* right wall */
        quad(556.0f, 0, 0, 0, 0, 559.2f, 0, 548.8f, 0, red);      /* left wall */
        orx_material em = {};
        em.type = ORX_MAT_DIFFUSE_EMITTER;
        for (int k = 0; k < 3; k++) {
            em.Kd[k] = 1.0f;
            em.power[k] = pw[k];
        }
        em.inverse_area = inv_area;
        em.texture = -1;
        m_mats.push_back(em);
        quad(lp[0], lp[1], lp[2], lv1[0], lv1[1], lv1[2], lv2[0], lv2[1], lv2[2], (uint32_t)m_mats.size() - 1);
    }
    orx_scene getFlatScene() const override {
        orx_scene s = {};
        s.n_quads = (uint32_t)m_qmat.size();
        s.quads = m_quads.data();
        s.quad_material = m_qmat.data();
        s.n_materials = (uint32_t)m_mats.size();
        s.materials = m_mats.data();
        s.n_lights = (uint32_t)m_lights.size();
        s.lights = m_lights.data();
        getSceneAABB(s.aabb_min, s.aabb_max);
        return s;
    }
    const char* getSceneName() const override { return "Cornell"; }
    Camera getDefaultCamera() const override { /* Cornell.cpp:199-207 */
        const float eye[3] = {278.0f, 273.0f, -850.0f}, at[3] = {278.0f, 273.0f, 0.0f}, up[3] = {0.0f, 1.0f, 0.0f};
        return Camera(eye, at, up, 35.0f, 35.0f, 0.0f);
    }
    void getSceneAABB(float mn[3], float mx[3]) const override { /* Cornell.cpp:28-31 */
        const float hi[3] = {556.0f, 548.85f, 559.2f};
        for (int k = 0; k < 3; k++) {
            mn[k] = -5.0f;
            mx[k] = hi[k] + 5.0f;
        }
    }

private:
    uint32_t material(int32_t type, float r, float g, float b) {
        orx_material m = {};
        m.type = type;
        m.Kd[0] = r;
        m.Kd[1] = g;
        m.Kd[2] = b;
        m.ior = 1.0f;
        m.exponent = 1.0f;
        m.texture = -1;
        m_mats.push_back(m);
        return (uint32_t)m_mats.size() - 1;
    }
    void quad(float ax, float ay, float az, float ux, float uy, float uz, float vx, float vy, float vz, uint32_t mat) {
        const float q[9] = {ax, ay, az, ux, uy, uz, vx, vy, vz};
        m_quads.insert(m_quads.end(), q, q + 9);
        m_qmat.push_back(mat);
    }
    std::vector<float> m_quads;
    std::vector<uint32_t> m_qmat;
    std::vector<orx_material> m_mats;
    std::vector<orx_light> m_lights;
};

int main(int argc, char** argv) {
    const char* method = "ppm";
    const char* out = nullptr;
    unsigned W = 32, H = 32, P = 64, iters = 2, seed = 1645301512u;
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "--print-camera") && i + 2 < argc) {
            Camera c = Cornell().getDefaultCamera();
            c.setAspectRatio((float)std::atoi(argv[i + 1]) / (float)std::atoi(argv[i + 2]));
            std::printf("%.9g %.9g %.9g\n", c.hfov, c.vfov, Cornell().getSceneInitialPPMRadiusEstimate());
            return 0;
        }
        if (!std::strcmp(argv[i], "--print-emitted") && i + 1 < argc) {
            /* the process-wide constant before and after setConfig (no device needed) */
            const unsigned before = OptixRenderer::EMITTED_PHOTONS_PER_ITERATION;
            OptixRenderer r;
            orx_config cfg;
            orx_default_config(&cfg);
            cfg.photon_launch_width = cfg.photon_launch_height = (unsigned)std::atoi(argv[i + 1]);
            r.setConfig(cfg);
            std::printf("%u %u\n", before, OptixRenderer::EMITTED_PHOTONS_PER_ITERATION);
            return 0;
        }
        if (i + 1 >= argc) break;
        if (!std::strcmp(argv[i], "--method")) method = argv[++i];
        else if (!std::strcmp(argv[i], "--width")) W = (unsigned)std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--height")) H = (unsigned)std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--photon-launch")) P = (unsigned)std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--iterations")) iters = (unsigned)std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--seed")) seed = (unsigned)std::strtoul(argv[++i], nullptr, 10);
        else if (!std::strcmp(argv[i], "--out")) out = argv[++i];
    }
    const RenderMethod::E m = !std::strcmp(method, "pt")    ? RenderMethod::PATH_TRACING
                              : !std::strcmp(method, "vcm") ? RenderMethod::BIDIRECTIONAL_PATH_TRACING
                                                            : RenderMethod::PROGRESSIVE_PHOTON_MAPPING;
    try {
        Cornell scene;
        OptixRenderer renderer;
        orx_config cfg;
        orx_default_config(&cfg);
        cfg.photon_launch_width = cfg.photon_launch_height = P;
        cfg.seed = seed;
        renderer.setConfig(cfg);
        renderer.initialize(ComputeDevice(0));
        renderer.initScene(scene);
        Camera cam = scene.getDefaultCamera();
        cam.setAspectRatio((float)W / (float)H);
        const double alpha = 2.0 / 3.0;
        RenderServerRenderRequestDetails details(cam, scene.getSceneName(), m, W, H, alpha);
        double radius = scene.getSceneInitialPPMRadiusEstimate();
        for (unsigned long long it = 0; it < iters; it++) {
            renderer.renderNextIteration(it, it, (float)radius, true, details);
            /* StandaloneRenderManager.cpp:105-107 */
            const double r2 = radius * radius * ((double)it + alpha) / ((double)it + 1.0);
            radius = std::sqrt(r2);
        }
        std::vector<float> img(renderer.getScreenBufferSizeBytes() / sizeof(float));
        renderer.getOutputBuffer(img.data());
        if (renderer.getWidth() != W || renderer.getHeight() != H) throw std::runtime_error("size mismatch");
        if (out) {
            FILE* f = std::fopen(out, "wb");
            if (!f || std::fwrite(img.data(), sizeof(float), img.size(), f) != img.size())
                throw std::runtime_error("cannot write output");
            std::fclose(f);
        }
        double sum = 0;
        for (float v : img) sum += v;
        std::printf("ok %s %ux%u photons %u iterations %u mean %.9g\n", method, W, H,
                    OptixRenderer::EMITTED_PHOTONS_PER_ITERATION, iters, sum / (double)img.size());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}

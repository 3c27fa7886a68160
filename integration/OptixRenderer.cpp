/*
 * OptixRenderer.cpp — orx-backed replacement of the reference's render core
 * (RenderEngine/renderer/OptixRenderer.cpp): the shim INTEGRATION.md describes,
 * compiled here against OptixRenderer.h (the restated interface) and linked
 * with liborx.so.  Every method keeps the reference's semantics and errors:
 *   OptixRenderer::initialize   throws on a second call (OptixRenderer.cpp:113-118)
 *   initScene                   throws before initialize and on a light-less scene (:436-447)
 *   renderNextIteration         resize + RNG re-init on a W/H change, accumulator zeroed at
 *                               localIterationNumber == 0, createOutput ignored (:507-821)
 *   getOutputBuffer             W*H*3 floats, running sum, caller-owned memory (:860-865)
 */
#include "OptixRenderer.h"

#include <cmath>
#include <stdexcept>

unsigned int OptixRenderer::EMITTED_PHOTONS_PER_ITERATION = 1024u * 1024u;
unsigned int OptixRenderer::s_liveRenderers = 0;

static void check(orx_renderer* r, orx_status s) {
    if (s != ORX_OK) throw std::runtime_error(r ? orx_last_error(r) : "orx: invalid renderer");
}

Camera::Camera(const float e[3], const float l[3], const float u[3], float h, float v, float a, AspectRatioMode m)
    : hfov(h), vfov(v), aperture(a), aspectRatioMode(m) {
    for (int k = 0; k < 3; k++) {
        eye[k] = e[k];
        lookat[k] = l[k];
        up[k] = u[k];
    }
}

/* Camera.cpp:294-318 in float (tan/atan of the float argument in double, as the host math does) */
void Camera::setAspectRatio(float ratio) {
    const float d2r = (float)M_PI / 180.0f, r2d = 180.0f / (float)M_PI;
    const float in = aspectRatioMode == KeepHorizontal ? hfov : vfov;
    const float real = aspectRatioMode == KeepHorizontal ? 1.0f / ratio : ratio;
    const float t = (float)std::tan((double)((0.5f * in) * d2r));
    const float out = (2.0f * (float)std::atan((double)(real * t))) * r2d;
    if (aspectRatioMode == KeepHorizontal)
        vfov = out;
    else
        hfov = out;
}

float IScene::getSceneInitialPPMRadiusEstimate() const {
    float mn[3], mx[3];
    getSceneAABB(mn, mx);
    const float ex = mx[0] - mn[0], ey = mx[1] - mn[1], ez = mx[2] - mn[2];
    const float volume = (ex * ey) * ez;
    const float cube = (float)std::pow((double)volume, 1.0 / 3.0);
    const float A = (6.0f * cube) * cube;
    return (float)((double)A * 3.94e-6);
}

OptixRenderer::OptixRenderer() : m_orx(nullptr), m_initialized(false) { orx_default_config(&m_cfg); }

OptixRenderer::~OptixRenderer() {
    orx_destroy(m_orx);
    if (m_initialized) s_liveRenderers--;
}

void OptixRenderer::setConfig(const orx_config& cfg) {
    if (m_initialized) throw std::runtime_error("OptixRenderer::setConfig after initialize");
    const unsigned long long launch = (unsigned long long)cfg.photon_launch_width * cfg.photon_launch_height;
    if (launch == 0 || launch > 0xFFFFFFFFull)
        throw std::invalid_argument("OptixRenderer::setConfig: photon launch must hold 1 .. 2^32-1 photons");
    if (s_liveRenderers > 0 && launch != EMITTED_PHOTONS_PER_ITERATION)
        throw std::invalid_argument("OptixRenderer::setConfig: EMITTED_PHOTONS_PER_ITERATION is process-wide and an "
                                    "initialized renderer uses a different photon launch");
    m_cfg = cfg;
    EMITTED_PHOTONS_PER_ITERATION = (unsigned int)launch;
}

void OptixRenderer::initialize(const ComputeDevice& device) {
    if (m_initialized) throw std::runtime_error("ERROR: Multiple OptixRenderer::initialize!");
    const unsigned int launch = m_cfg.photon_launch_width * m_cfg.photon_launch_height;
    if (s_liveRenderers > 0 && launch != EMITTED_PHOTONS_PER_ITERATION)
        throw std::invalid_argument("OptixRenderer::initialize: another initialized renderer uses a different "
                                    "photon launch (EMITTED_PHOTONS_PER_ITERATION is process-wide)");
    orx_renderer* r = nullptr;
    if (orx_create(device.getDeviceId(), &m_cfg, &r) != ORX_OK) {
        orx_destroy(r);
        throw std::runtime_error("OptixRenderer::initialize: no usable device");
    }
    m_orx = r;
    m_initialized = true;
    s_liveRenderers++;
    EMITTED_PHOTONS_PER_ITERATION = orx_emitted_photons_per_iteration(r); /* this renderer's launch */
}

void OptixRenderer::initScene(IScene& scene) {
    if (!m_initialized) throw std::runtime_error("Cannot initialize scene before OptixRenderer.");
    const orx_scene flat = scene.getFlatScene();
    check(m_orx, orx_init_scene(m_orx, &flat));
}

void OptixRenderer::renderNextIteration(unsigned long long iterationNumber, unsigned long long localIterationNumber,
                                        float PPMRadius, bool createOutput,
                                        const RenderServerRenderRequestDetails& d) {
    if (!m_initialized) throw std::runtime_error("Traced before OptixRenderer was initialized.");
    const Camera& c = d.getCamera();
    orx_request req = {};
    for (int k = 0; k < 3; k++) {
        req.camera.eye[k] = c.eye[k];
        req.camera.lookat[k] = c.lookat[k];
        req.camera.up[k] = c.up[k];
    }
    req.camera.hfov = c.hfov;
    req.camera.vfov = c.vfov;
    req.camera.aperture = c.aperture;
    req.method = (int32_t)d.getRenderMethod(); /* RenderMethod::E order == orx_method */
    req.width = d.getWidth();
    req.height = d.getHeight();
    req.ppm_alpha = d.getPPMAlpha();
    check(m_orx, orx_render_next_iteration(m_orx, iterationNumber, localIterationNumber, PPMRadius,
                                           createOutput ? 1 : 0, &req));
}

void OptixRenderer::getOutputBuffer(void* data) {
    check(m_orx, orx_get_output(m_orx, (float*)data, orx_output_bytes(m_orx)));
}

unsigned int OptixRenderer::getWidth() const { return orx_width(m_orx); }
unsigned int OptixRenderer::getHeight() const { return orx_height(m_orx); }
unsigned int OptixRenderer::getScreenBufferSizeBytes() const { return (unsigned int)orx_output_bytes(m_orx); }

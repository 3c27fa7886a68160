/*
 * OptixRenderer.h — the public interface of the reference's render core class
 * (RenderEngine/renderer/OptixRenderer.h:21-43), restated with the minimal
 * companion types its signatures name (ComputeDevice, IScene, Camera,
 * RenderMethod, RenderServerRenderRequestDetails), so that the orx-backed shim
 * a maintainer drops into the reference (OptixRenderer.cpp next to this file,
 * the binding INTEGRATION.md describes) is compiled and run here against
 * liborx.so.  It is not the reference's header: only the method names,
 * parameters and semantics callers rely on are kept (StandaloneRenderManager.cpp
 * :60, :86, :104, :122, :155; RenderServerRenderer.cpp:58, :154, :170-172).
 */
#pragma once

#include <string>

#include "orx.h"

/* ComputeDevice (RenderEngine/ComputeDevice.h): the CUDA ordinal, here a HIP device index. */
class ComputeDevice {
public:
    explicit ComputeDevice(int id = 0) : m_id(id) {}
    int getDeviceId() const { return m_id; }

private:
    int m_id;
};

/* RenderMethod::E (renderer/RenderMethod.h:13-19); same order as orx_method. */
namespace RenderMethod {
enum E { PATH_TRACING = 0, BIDIRECTIONAL_PATH_TRACING = 1, PROGRESSIVE_PHOTON_MAPPING = 2 };
}

/* Camera inputs (renderer/Camera.h:72-79) and Camera::setAspectRatio (Camera.cpp:294-318). */
class Camera {
public:
    enum AspectRatioMode { KeepVertical, KeepHorizontal };
    Camera(const float eye[3], const float lookat[3], const float up[3], float hfov, float vfov, float aperture,
           AspectRatioMode mode = KeepVertical);
    void setAspectRatio(float ratio);
    float eye[3], lookat[3], up[3];
    float hfov, vfov, aperture;
    AspectRatioMode aspectRatioMode;
};

/* RenderServerRenderRequestDetails (clientserver/RenderServerRenderRequestDetails.h:15-33). */
class RenderServerRenderRequestDetails {
public:
    RenderServerRenderRequestDetails(const Camera& camera, const std::string& sceneName, RenderMethod::E method,
                                     unsigned int width, unsigned int height, double ppmAlpha)
        : m_camera(camera), m_sceneName(sceneName), m_method(method), m_width(width), m_height(height),
          m_alpha(ppmAlpha) {}
    const Camera& getCamera() const { return m_camera; }
    const std::string& getSceneName() const { return m_sceneName; }
    RenderMethod::E getRenderMethod() const { return m_method; }
    unsigned int getWidth() const { return m_width; }
    unsigned int getHeight() const { return m_height; }
    double getPPMAlpha() const { return m_alpha; }

private:
    Camera m_camera;
    std::string m_sceneName;
    RenderMethod::E m_method;
    unsigned int m_width, m_height;
    double m_alpha;
};

/* IScene (scene/IScene.h:16-29).  getSceneRootGroup(optix::Context&) becomes
 * getFlatScene(): the geometry as plain arrays (the one API change). */
class IScene {
public:
    virtual ~IScene() {}
    virtual orx_scene getFlatScene() const = 0;
    virtual const char* getSceneName() const = 0;
    virtual Camera getDefaultCamera() const = 0;
    virtual void getSceneAABB(float mn[3], float mx[3]) const = 0;
    /* IScene.cpp:51-59: A * 3.94e-6, A = 6 * cbrt(V)^2 over the scene AABB */
    float getSceneInitialPPMRadiusEstimate() const;
};

/* OptixRenderer (renderer/OptixRenderer.h:21-43) */
class OptixRenderer {
public:
    OptixRenderer();
    ~OptixRenderer();
    void initialize(const ComputeDevice& device);
    void initScene(IScene& scene);
    void renderNextIteration(unsigned long long iterationNumber, unsigned long long localIterationNumber,
                             float PPMRadius, bool createOutput, const RenderServerRenderRequestDetails& details);
    void getOutputBuffer(void* data);
    unsigned int getWidth() const;
    unsigned int getHeight() const;
    unsigned int getScreenBufferSizeBytes() const;
    /* PHOTON_LAUNCH_WIDTH * PHOTON_LAUNCH_HEIGHT (OptixRenderer.h:43).  The reference compiles
     * the launch size in, so this is process-wide: it follows the photon launch of the last
     * setConfig (1024 x 1024 by default) and callers read it as before
     * (DistributedApplication.cpp:133-134).  Not const, since setConfig sets it. */
    static unsigned int EMITTED_PHOTONS_PER_ITERATION;

    /* not in the reference: the config.h constants the engine otherwise compiles in
     * (photon launch size, seed, ...), before initialize().  Throws std::invalid_argument when
     * the photon launch differs from the one of a renderer that is already initialized in this
     * process (EMITTED_PHOTONS_PER_ITERATION can hold only one value, as in the reference) */
    void setConfig(const orx_config& cfg);

private:
    static unsigned int s_liveRenderers; /* initialized, not yet destroyed */
    orx_renderer* m_orx;
    orx_config m_cfg;
    bool m_initialized;
};

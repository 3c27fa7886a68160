"""ctypes mirror of include/orx.h (the C-ABI drop-in boundary).

Pure layout definitions: no library is loaded here.  `renderer.py` binds
these to liborx.so (the HIP product); the test-suite binds the same
structures to the CPU oracle so both are driven through identical calls.
"""
import ctypes as C

ORX_OK = 0
ORX_ERR_INVALID_ARGUMENT = 1
ORX_ERR_STATE = 2
ORX_ERR_DEVICE = 3
ORX_ERR_NO_LIGHTS = 4
ORX_ERR_GRID_TOO_LARGE = 5
ORX_ERR_OUT_OF_MEMORY = 6
ORX_ERR_UNSUPPORTED = 7

# RenderMethod::E (RenderEngine/renderer/RenderMethod.h:13-19)
PATH_TRACING = 0
VCM_BIDIRECTIONAL_PATH_TRACING = 1
PROGRESSIVE_PHOTON_MAPPING = 2

# orx_config.photon_map (config.h ACCELERATION_STRUCTURE)
PHOTON_MAP_UNIFORM_GRID = 0
PHOTON_MAP_STOCHASTIC_HASH = 1
PHOTON_MAP_KD_TREE = 2

MAT_DIFFUSE = 0
MAT_DIFFUSE_EMITTER = 1
MAT_MIRROR = 2
MAT_GLASS = 3
MAT_GLOSSY = 4
MAT_TEXTURE = 5

LIGHT_AREA = 0
LIGHT_POINT = 1
LIGHT_SPOT = 2

BUF_RNG = 0
BUF_HITPOINTS = 1
BUF_PHOTONS = 2
BUF_GRID_OFFSETS = 3
BUF_INDIRECT = 4
BUF_DIRECT = 5
BUF_OUTPUT = 6
BUF_PHOTON_SLOTS = 7
BUF_DEBUG_VISITED = 8
BUF_VCM_VERTEX_COUNT = 9
BUF_VCM_VERTICES = 10
BUF_VCM_SPLAT = 11
BUF_VCM_CAMERA = 12
BUF_KD_TREE = 13
BUF_VOLUMETRIC = 14
BUF_VOLUMETRIC_PHOTONS = 15

# RadiancePRD.h:30-35 flag bits
PRD_HIT_EMITTER = 1 << 31
PRD_ERROR = 1 << 30
PRD_MISS = 1 << 29
PRD_HIT_SPECULAR = 1 << 28
PRD_HIT_NON_SPECULAR = 1 << 27
PRD_PATH_TRACING = 1 << 26

F3 = C.c_float * 3


class OrxCamera(C.Structure):
    _fields_ = [("eye", F3), ("lookat", F3), ("up", F3),
                ("hfov", C.c_float), ("vfov", C.c_float), ("aperture", C.c_float)]


class OrxRequest(C.Structure):
    _fields_ = [("camera", OrxCamera), ("method", C.c_int32), ("width", C.c_uint32),
                ("height", C.c_uint32), ("ppm_alpha", C.c_double)]


class OrxMaterial(C.Structure):
    _fields_ = [("type", C.c_int32), ("Kd", F3), ("Ks", F3), ("Kr", F3), ("Kt", F3),
                ("ior", C.c_float), ("exponent", C.c_float), ("power", F3),
                ("inverse_area", C.c_float), ("texture", C.c_int32)]


class OrxTexture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("rgba", C.POINTER(C.c_uint8)),
                ("normal_width", C.c_uint32), ("normal_height", C.c_uint32),
                ("normal_rgba", C.POINTER(C.c_uint8))]


class OrxLight(C.Structure):
    _fields_ = [("type", C.c_int32), ("power", F3), ("position", F3), ("v1", F3), ("v2", F3),
                ("direction", F3), ("angle", C.c_float)]


class OrxScene(C.Structure):
    _fields_ = [
        ("n_quads", C.c_uint32), ("quads", C.POINTER(C.c_float)), ("quad_material", C.POINTER(C.c_uint32)),
        ("n_spheres", C.c_uint32), ("spheres", C.POINTER(C.c_float)), ("sphere_material", C.POINTER(C.c_uint32)),
        ("n_vertices", C.c_uint32), ("vertices", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
        ("n_triangles", C.c_uint32), ("triangles", C.POINTER(C.c_uint32)),
        ("triangle_material", C.POINTER(C.c_uint32)),
        ("n_materials", C.c_uint32), ("materials", C.POINTER(OrxMaterial)),
        ("n_lights", C.c_uint32), ("lights", C.POINTER(OrxLight)),
        ("aabb_min", F3), ("aabb_max", F3),
        ("texcoords", C.POINTER(C.c_float)), ("tangents", C.POINTER(C.c_float)),
        ("bitangents", C.POINTER(C.c_float)),
        ("n_textures", C.c_uint32), ("textures", C.POINTER(OrxTexture)),
        ("n_media", C.c_uint32), ("media", C.POINTER(C.c_float)),
    ]


class OrxConfig(C.Structure):
    _fields_ = [("photon_launch_width", C.c_uint32), ("photon_launch_height", C.c_uint32),
                ("max_photon_deposits", C.c_uint32), ("photon_grid_max_size", C.c_uint32),
                ("max_photon_trace_depth", C.c_uint32), ("max_radiance_trace_depth", C.c_uint32),
                ("vcm_max_path_length", C.c_uint32), ("seed", C.c_uint32),
                ("debug_counters", C.c_uint32), ("gather_variant", C.c_uint32), ("photon_map", C.c_uint32),
                ("enable_media", C.c_uint32), ("volumetric_photons", C.c_uint32), ("reserved", C.c_uint32 * 3)]


class OrxStats(C.Structure):
    _fields_ = [("grid_size", C.c_uint32 * 3), ("cell_size", C.c_float), ("world_origin", F3),
                ("valid_photons", C.c_uint32), ("num_cells", C.c_uint32),
                ("photons_visited", C.c_uint64), ("cells_visited", C.c_uint64),
                ("photons_visited_total", C.c_uint64), ("cells_visited_total", C.c_uint64),
                ("valid_photons_total", C.c_uint64), ("vcm_shadow_rays", C.c_uint32), ("vcm_shadow_overflow", C.c_uint32),
                ("timed_iterations", C.c_uint32), ("bvh_stack_entries", C.c_uint32), ("pass_ms", C.c_float * 16),
                ("vcm_light_connections", C.c_uint32), ("vcm_light_inplace", C.c_uint32)]


PASS_NAMES = ["ppm_eye", "ppm_photon", "grid_hash", "grid_scan", "grid_scatter", "ppm_gather", "ppm_direct_output",
              "pt", "vcm_light", "vcm_camera", "vcm_shadow"]


def default_config(**overrides):
    """orx_default_config values (config.h / OptixRenderer.cpp:38-61)."""
    c = OrxConfig()
    c.photon_launch_width = 1024
    c.photon_launch_height = 1024
    c.max_photon_deposits = 4
    c.photon_grid_max_size = 100 * 100 * 100
    c.max_photon_trace_depth = 7
    c.max_radiance_trace_depth = 9
    c.vcm_max_path_length = 10
    c.seed = 0
    c.debug_counters = 1
    c.volumetric_photons = 200000  # NUM_VOLUMETRIC_PHOTONS (config.h:35)
    for k, v in overrides.items():
        setattr(c, k, v)
    return c


def declare_common(lib, prefix):
    """Attach argtypes/restype for the entry points shared by liborx (prefix
    'orx') and the oracle (prefix 'orc')."""
    vp = C.c_void_p
    f = getattr(lib, prefix + "_init_scene")
    f.argtypes, f.restype = [vp, C.POINTER(OrxScene)], C.c_int
    f = getattr(lib, prefix + "_render_next_iteration")
    f.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_float, C.c_int, C.POINTER(OrxRequest)]
    f.restype = C.c_int
    f = getattr(lib, prefix + "_get_output")
    f.argtypes, f.restype = [vp, C.c_void_p, C.c_size_t], C.c_int
    f = getattr(lib, prefix + "_read_buffer")
    f.argtypes, f.restype = [vp, C.c_int32, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)], C.c_int
    f = getattr(lib, prefix + "_get_stats")
    f.argtypes, f.restype = [vp, C.POINTER(OrxStats)], C.c_int
    f = getattr(lib, prefix + "_last_error")
    f.argtypes, f.restype = [vp], C.c_char_p
    f = getattr(lib, prefix + "_destroy")
    f.argtypes, f.restype = [vp], None

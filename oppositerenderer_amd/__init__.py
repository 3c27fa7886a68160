"""oppositerenderer_amd — MI355X-native progressive photon mapping / path
tracing / VCM render core that drops in behind OppositeRenderer's
OptixRenderer API (include/orx.h)."""
from . import _abi  # noqa: F401
from .scenes import Camera, Scene, cornell, cornell_small, scene_by_name  # noqa: F401

__all__ = ["Camera", "Scene", "cornell", "cornell_small", "scene_by_name"]

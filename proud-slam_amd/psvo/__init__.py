"""psvo — MI355X-native sparse-voxel-octree renderer for the Proud-SLAM
render-and-optimise hot path.

Put `proud-slam_amd/` on sys.path; then `import grid` is the drop-in for the
reference's `grid` extension and `psvo.render_helpers` / `psvo.voxel_helpers`
/ `psvo.criterion` / `psvo.decoder` / `psvo.octree` mirror the reference's
modules of the same role.
"""
from . import _lib  # noqa: F401

__all__ = ["_lib", "octree", "voxel_helpers", "render_helpers", "criterion", "decoder", "synthetic", "dist"]


def version():
    return _lib.lib().psvo_version().decode()

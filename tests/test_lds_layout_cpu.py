"""The D = 256 attention LDS image layout (attention.hip Img<256>, slab images) is bank-conflict
free for both fragment reads on gfx950's lane groups: scripts/diag/slab_swizzle_check.py."""

import importlib.util
import os

_P = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts", "diag",
                  "slab_swizzle_check.py")


def test_slab_images_conflict_free():
    spec = importlib.util.spec_from_file_location("slab_swizzle_check", _P)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    for rows in (32, 64):
        m.check(rows)

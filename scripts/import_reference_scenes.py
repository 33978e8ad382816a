#!/usr/bin/env python3
"""Copies the reference's scene INPUT DATA into scenes/ (run here only;
/root/reference is absent on the GPU box, so the copies are committed):
  scenes/killeroo-simple.pbrt       BASELINE config 1 (reference scenes/killeroo-simple.pbrt)
  scenes/geometry/killeroo.pbrt     its Loop-subdivision control mesh (reference scenes/geometry/)
  scenes/lamp/lamp.pbrt             the reference's one portal scene (scenes/blender/lamp/out/lamp.pbrt:
                                    two axis-2 portals, one '+'-facing, plymesh, matte + metal)
  scenes/lamp/meshes/00001/*.ply    its meshes (binary little-endian PLY, byte-identical copies)
Scene files are renderer inputs (fixtures), not source; a provenance comment is
prepended to each text file."""
import os
import shutil

SRC = "/root/reference/scenes"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scenes")

TEXT = [("killeroo-simple.pbrt", "killeroo-simple.pbrt"),
        ("geometry/killeroo.pbrt", "geometry/killeroo.pbrt"),
        ("blender/lamp/out/lamp.pbrt", "lamp/lamp.pbrt")]
BINARY = [("blender/lamp/out/meshes/00001/%s.ply" % m, "lamp/meshes/00001/%s.ply" % m)
          for m in ("Base_mat0", "Lampshade_mat0", "Leg_mat0", "Room_mat1", "Room_mat2")]

for rel, dst in TEXT:
    out = os.path.join(DST, dst)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(os.path.join(SRC, rel)) as f, open(out, "w") as g:
        g.write(f"# scene input data from the reference's scenes/{rel} "
                "(copied by scripts/import_reference_scenes.py)\n")
        g.write(f.read())
    print("wrote", os.path.normpath(out))
for rel, dst in BINARY:
    out = os.path.join(DST, dst)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    shutil.copyfile(os.path.join(SRC, rel), out)
    print("wrote", os.path.normpath(out))

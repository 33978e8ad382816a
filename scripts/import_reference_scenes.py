#!/usr/bin/env python3
"""Copies the reference's scene INPUT DATA into scenes/ (run here only;
/root/reference is absent on the GPU box, so the copies are committed):
  scenes/killeroo-simple.pbrt       BASELINE config 1 (reference scenes/killeroo-simple.pbrt)
  scenes/geometry/killeroo.pbrt     its Loop-subdivision control mesh (reference scenes/geometry/)
  scenes/lamp/lamp.pbrt             the reference's one portal scene (scenes/blender/lamp/out/lamp.pbrt:
                                    two axis-2 portals, one '+'-facing, plymesh, matte + metal)
  scenes/lamp/meshes/00001/*.ply    its meshes (binary little-endian PLY, byte-identical copies)
  scenes/creeper/creeper.pbrt       scenes/blender/creeper/out/creeper.pbrt: DiffuseAreaLight on an axis-1
                                    aaplane (carrying unused "portalData" with five '+' portals), a point
                                    light, Scale -1 1 1 before LookAt, DirectLighting
  scenes/creeper/sandbox.pbrt       scenes/blender/creeper/out/sandbox.pbrt: PortalArealight under a rotated
                                    Transform, five axis-2 '+' portals, strategy projection, DirectLighting
  scenes/creeper/test00001.pbrt     scenes/blender/creeper/out/test00001.pbrt: path, trianglemesh emitter
  scenes/creeper/meshes/00001/*.ply their meshes (byte-identical copies)
  scenes/lamp/test00001.pbrt        scenes/blender/lamp/out/test00001.pbrt: DiffuseAreaLight on an aaplane,
                                    metal, DirectLighting (same meshes as lamp.pbrt)
  scenes/spotlight/test00001.pbrt   scenes/blender/spotlight/out/test00001.pbrt: DirectLighting "one", two
                                    diffuse trianglemesh lights, one of them an empty mesh ("point P" [])
  scenes/spotlight/arealight.pbrt   scenes/blender/spotlight/out/arealight.pbrt: path maxdepth 10, aaplane
                                    with the old loX/hiX parameters (lo = hi = 0, as in creeper)
  scenes/window_portal_eq/test00001.pbrt  scenes/blender/window_portal_eq/out/test00001.pbrt: DirectLighting
                                    "one", two diffuse lights
  scenes/{spotlight,window_portal_eq}/meshes/00001/*.ply  the meshes they name (byte-identical copies)
Scene files are renderer inputs (fixtures), not source; a provenance comment is
prepended to each text file."""
import os
import shutil

SRC = "/root/reference/scenes"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scenes")

TEXT = [("killeroo-simple.pbrt", "killeroo-simple.pbrt"),
        ("geometry/killeroo.pbrt", "geometry/killeroo.pbrt"),
        ("blender/lamp/out/lamp.pbrt", "lamp/lamp.pbrt"),
        ("blender/creeper/out/creeper.pbrt", "creeper/creeper.pbrt"),
        ("blender/creeper/out/sandbox.pbrt", "creeper/sandbox.pbrt"),
        ("blender/creeper/out/test00001.pbrt", "creeper/test00001.pbrt"),
        ("blender/lamp/out/test00001.pbrt", "lamp/test00001.pbrt"),
        ("blender/spotlight/out/test00001.pbrt", "spotlight/test00001.pbrt"),
        ("blender/spotlight/out/arealight.pbrt", "spotlight/arealight.pbrt"),
        ("blender/window_portal_eq/out/test00001.pbrt", "window_portal_eq/test00001.pbrt")]
BINARY = [("blender/lamp/out/meshes/00001/%s.ply" % m, "lamp/meshes/00001/%s.ply" % m)
          for m in ("Base_mat0", "Lampshade_mat0", "Leg_mat0", "Room_mat1", "Room_mat2")]
BINARY += [("blender/creeper/out/meshes/00001/%s.ply" % m, "creeper/meshes/00001/%s.ply" % m)
           for m in ("Cube_mat0", "Ground_mat0", "creeper.001_mat0", "creeper_mat0")]
BINARY += [("blender/spotlight/out/meshes/00001/%s.ply" % m, "spotlight/meshes/00001/%s.ply" % m)
           for m in ("shade_mat1", "Suzanne_mat0")]
BINARY += [("blender/window_portal_eq/out/meshes/00001/%s.ply" % m, "window_portal_eq/meshes/00001/%s.ply" % m)
           for m in ("Cube_mat1", "Suzanne_mat0")]

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

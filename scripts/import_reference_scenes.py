#!/usr/bin/env python3
"""Copies the reference's killeroo scene INPUT DATA into scenes/ (run here
only; /root/reference is absent on the GPU box, so the copies are committed):
  scenes/killeroo-simple.pbrt       BASELINE config 1 (reference scenes/killeroo-simple.pbrt)
  scenes/geometry/killeroo.pbrt     its Loop-subdivision control mesh (reference scenes/geometry/)
Scene files are renderer inputs (fixtures), not source; a provenance comment is
prepended to each."""
import os

SRC = "/root/reference/scenes"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scenes")

for rel in ("killeroo-simple.pbrt", "geometry/killeroo.pbrt"):
    out = os.path.join(DST, rel)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(os.path.join(SRC, rel)) as f, open(out, "w") as g:
        g.write(f"# scene input data from the reference's scenes/{rel} "
                "(copied by scripts/import_reference_scenes.py)\n")
        g.write(f.read())
    print("wrote", os.path.normpath(out))

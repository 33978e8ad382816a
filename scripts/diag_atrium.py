"""Diagnostic: render a 12-copy config-5 atrium at 64x36x4 with
PT_SYNC_CHECK=1 so a device fault names its kernel and bounce."""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pbrt-v3-light-portals_amd"))
import ptgpu  # noqa: E402

out = os.path.join(os.environ.get("TMPDIR", "/tmp"), "diag_atrium.pbrt")
subprocess.check_call([sys.executable, os.path.join(REPO, "scripts", "make_atrium.py"), out, "--copies",
                       sys.argv[1] if len(sys.argv) > 1 else "12"])
txt = open(out).read()
txt = re.sub(r'Include "([^"]+)"', lambda m: 'Include "%s/scenes/%s"' % (REPO, m.group(1)), txt)
txt = re.sub(r'"integer xresolution" \[\d+\]', '"integer xresolution" [64]', txt)
txt = re.sub(r'"integer yresolution" \[\d+\]', '"integer yresolution" [36]', txt)
txt = re.sub(r'"integer pixelsamples" \[\d+\]', '"integer pixelsamples" [4]', txt)
open(out, "w").write(txt)
hs = ptgpu.HostScene(out)
sc = ptgpu.Scene(hs)
print("scene ok", flush=True)
try:
    img, st = sc.render()
    print("render ok", img.mean(), st, flush=True)
except ptgpu.PtError as e:
    print("render failed:", e, flush=True)
    sys.exit(3)

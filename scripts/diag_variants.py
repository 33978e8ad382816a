"""Diagnostic: build config-5 atrium variants (12 copies, 64x36x4) and render
the one named on the command line with PT_SYNC_CHECK=1.
  portal   as generated (skylight portal, strategy "portal")
  light    strategy "light" (no portal sampling)
  quad     emitter as a diffuse trianglemesh quad (no aaplane / portal)
  room     no killeroos (portal strategy)"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pbrt-v3-light-portals_amd"))
import ptgpu  # noqa: E402

which = sys.argv[1]
out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"diag_{which}.pbrt")
subprocess.check_call([sys.executable, os.path.join(REPO, "scripts", "make_atrium.py"), out, "--copies",
                       "0" if which == "room" else "12"])
txt = open(out).read()
txt = re.sub(r'Include "([^"]+)"', lambda m: 'Include "%s/scenes/%s"' % (REPO, m.group(1)), txt)
txt = re.sub(r'"integer xresolution" \[\d+\]', '"integer xresolution" [64]', txt)
txt = re.sub(r'"integer yresolution" \[\d+\]', '"integer yresolution" [36]', txt)
txt = re.sub(r'"integer pixelsamples" \[\d+\]', '"integer pixelsamples" [4]', txt)
if which == "light":
    txt = txt.replace('"string strategy" "portal"', '"string strategy" "light"')
if which == "quad":
    txt = re.sub(r'AreaLightSource "portal".*?Shape "aaplane"[^\n]*\n',
                 'AreaLightSource "diffuse" "rgb L" [30 29 27] "bool twosided" "true"\n'
                 '  Shape "trianglemesh" "integer indices" [0 1 2 2 3 0] "point P" '
                 '[-640 -1240 1500 640 -1240 1500 640 1240 1500 -640 1240 1500]\n', txt, flags=re.S)
open(out, "w").write(txt)
hs = ptgpu.HostScene(out)
if "--dry" in sys.argv:
    d = ptgpu._desc_prefix.from_address(hs.desc)
    print(which, "loads", d.n_prims, d.n_planes)
    sys.exit(0)
sc = ptgpu.Scene(hs)
print(which, "scene ok", flush=True)
try:
    img, st = sc.render()
    print(which, "render ok", img.mean(), st, flush=True)
except ptgpu.PtError as e:
    print(which, "render failed:", e, flush=True)
    sys.exit(3)

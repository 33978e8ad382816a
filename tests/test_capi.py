"""CPU checks of the drop-in boundary: the C-ABI library loads, exports every
symbol include/pt.h declares, and its host-only entry points behave (no GPU
compute is called here)."""
import ctypes
import os

import pytest

import ptgpu
from conftest import REPO


def test_library_exports_every_declared_symbol():
    names = ptgpu.exported_symbols()
    assert len(names) >= 20
    L = ptgpu.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_abi_version():
    assert ptgpu.lib().pt_abi_version() == 4


def test_pt_h_compiles_as_c():
    """The boundary header is plain C (no C++/torch types)."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "t.c")
        open(src, "w").write('#include "pt.h"\nint main(void){pt_scene_desc d; (void)d; return 0;}\n')
        subprocess.check_call(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(REPO, "include"), "-c",
                               src, "-o", os.path.join(d, "t.o")])


def test_errors_are_status_codes(tmp_path):
    p = tmp_path / "bad.pbrt"
    p.write_text('WorldBegin\nShape "cylinder"\nWorldEnd\n')
    with pytest.raises(ptgpu.PtError) as e:
        ptgpu.HostScene(str(p))
    assert e.value.status == 3  # PT_ERR_UNSUPPORTED
    with pytest.raises(ptgpu.PtError) as e:
        ptgpu.HostScene(str(tmp_path / "missing.pbrt"))
    assert e.value.status == 7  # PT_ERR_IO
    p.write_text('WorldBegin\nBogus "x"\nWorldEnd\n')
    with pytest.raises(ptgpu.PtError) as e:
        ptgpu.HostScene(str(p))
    assert e.value.status == 2  # PT_ERR_PARSE


def test_null_arguments_rejected():
    L = ptgpu.lib()
    assert L.pt_load_pbrt(None, None) == 1
    assert L.pt_render(None, None, None) == 1
    assert L.pt_scene_bvh(None, None, None, None, None) == 1
    assert L.pt_last_error()


def test_ctypes_mirror_matches_c_layout():
    """ptgpu's ctypes view of pt_scene_desc has the C layout (size and the
    offsets the tests read)."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "t.c")
        open(src, "w").write('#include <stdio.h>\n#include <stddef.h>\n#include "pt.h"\nint main(void){printf("%zu %zu %zu %zu",'
                             ' sizeof(pt_scene_desc), offsetof(pt_scene_desc, integrator), '
                             'offsetof(pt_scene_desc, n_spheres), sizeof(pt_material));return 0;}\n')
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(REPO, "include"), src, "-o", exe])
        got = [int(x) for x in subprocess.check_output([exe]).split()]
    import ctypes
    D = ptgpu.pt_scene_desc
    assert got == [ctypes.sizeof(D), D.integrator.offset, D.n_spheres.offset, ctypes.sizeof(ptgpu.pt_material)]

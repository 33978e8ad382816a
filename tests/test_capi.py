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
    assert ptgpu.lib().pt_abi_version() == 11


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
                             'offsetof(pt_scene_desc, n_spheres), sizeof(pt_material));'
                             'printf(" %zu %zu %zu", sizeof(pt_stats), offsetof(pt_stats, reduce_ms), sizeof(pt_light));'
                             'return 0;}\n')
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(REPO, "include"), src, "-o", exe])
        got = [int(x) for x in subprocess.check_output([exe]).split()]
    import ctypes
    D = ptgpu.pt_scene_desc
    assert got[:4] == [ctypes.sizeof(D), D.integrator.offset, D.n_spheres.offset, ctypes.sizeof(ptgpu.pt_material)]
    S = ptgpu.pt_stats
    assert got[4:] == [ctypes.sizeof(S), S.reduce_ms.offset, 168]  # tests index pt_light records as 42 int32


def test_bvh_host_capacities(tmp_path):
    """pt_build_bvh_host reports node and prim counts separately and rejects
    buffers smaller than them (a single 3-4-primitive leaf has n_nodes = 1 <
    n_prims)."""
    import ctypes
    import numpy as np
    from conftest import scene_variant
    hs = ptgpu.HostScene(scene_variant(tmp_path, res=(8, 8), spp=1))
    nodes, order = hs.bvh()
    assert sorted(order.tolist()) == list(range(len(order)))
    L = ptgpu.lib()
    n, m = ctypes.c_int32(), ctypes.c_int32()
    small = np.zeros(8 * len(nodes), np.uint32)
    o = np.zeros(len(order), np.int32)
    assert L.pt_build_bvh_host(hs.desc, ctypes.byref(n), small.ctypes.data, len(nodes) - 1, ctypes.byref(m),
                               None, 0) == 1
    assert L.pt_build_bvh_host(hs.desc, ctypes.byref(n), None, 0, ctypes.byref(m), o.ctypes.data,
                               len(order) - 1) == 1
    assert (n.value, m.value) == (len(nodes), len(order))


def test_multi_gpu_entry_points_reject_bad_arguments():
    """pt_init / the RCCL communicator entry points validate before touching
    a device (no GPU here: the device-less calls fail with a status)."""
    L = ptgpu.lib()
    assert L.pt_init(0, None) != 0
    assert L.pt_comm_create(0, 0, None, None) == 1
    assert L.pt_film_reduce(None, None, None, 0, None) == 1
    assert L.pt_render_frame_dist(None, None, None, None, None) == 1
    assert L.pt_scene_query(None, 0, None) == 1
    assert L.pt_shutdown() == 0

"""Film output formats (Film::WriteImage -> WriteImage, reference
src/core/imageio.cpp:81-122): EXR (half RGB, display/data windows), PFM,
PNG and TGA (8-bit after GammaCorrect).  Host only.

Each file is decoded here by an independent reader and compared with a
restatement of the reference's conversion: numpy's IEEE round-to-nearest-even
float16 for OpenEXR's half(float), and TO_BYTE = (uint8)Clamp(255 *
GammaCorrect(v) + 0.5, 0, 255) with glibc powf (pbrt.h:298-301,
imageio.cpp:91)."""
import ctypes
import struct
import zlib

import numpy as np
import pytest

import ptgpu

_libm = ctypes.CDLL("libm.so.6")
_libm.powf.restype = ctypes.c_float
_libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
F = np.float32


def to_byte(v):
    v = F(v)
    if v <= F(0.0031308):
        g = F(F(12.92) * v)
    else:
        g = F(F(F(1.055) * F(_libm.powf(v, F(F(1.0) / F(2.4))))) - F(0.055))
    x = F(F(F(255.0) * g) + F(0.5))
    x = F(0.0) if x < 0 else (F(255.0) if x > 255 else x)
    return int(x)


def _image(w=37, h=11, seed=0):
    rng = np.random.default_rng(seed)
    img = (rng.random((h, w, 3), dtype=np.float32) * 2.5).astype(np.float32)
    img[0, 0] = [0, 1e-5, 0.0031308]
    img[0, 1] = [70000.0, 65504.0, 65519.0]        # half overflow / max / rounds to max
    img[0, 2] = [6e-8, 3e-8, -2.0]                 # half subnormals, negative
    img[0, 3] = [1.0 + 2 ** -11, 1.0 + 3 * 2 ** -11, 0.5]  # ties to even
    return img


def read_exr(path):
    b = open(path, "rb").read()
    assert b[:4] == bytes([0x76, 0x2F, 0x31, 0x01]) and b[4] == 2
    pos, attrs = 8, {}
    while b[pos] != 0:
        e = b.index(0, pos)
        name = b[pos:e].decode()
        e2 = b.index(0, e + 1)
        typ = b[e + 1:e2].decode()
        size = struct.unpack_from("<i", b, e2 + 1)[0]
        attrs[name] = (typ, b[e2 + 5:e2 + 5 + size])
        pos = e2 + 5 + size
    pos += 1
    x0, y0, x1, y1 = struct.unpack("<4i", attrs["dataWindow"][1])
    disp = struct.unpack("<4i", attrs["displayWindow"][1])
    assert attrs["compression"][1] == b"\x00"
    chans, cp = [], attrs["channels"][1]
    i = 0
    while cp[i] != 0:
        e = cp.index(0, i)
        chans.append((cp[i:e].decode(), struct.unpack_from("<i", cp, e + 1)[0]))
        i = e + 17
    w, h = x1 - x0 + 1, y1 - y0 + 1
    offs = struct.unpack_from("<%dQ" % h, b, pos)
    out = np.zeros((h, w, len(chans)), np.float16)
    for k, o in enumerate(offs):
        y, n = struct.unpack_from("<ii", b, o)
        assert y == y0 + k and n == w * len(chans) * 2
        plane = np.frombuffer(b, np.float16, w * len(chans), o + 8).reshape(len(chans), w)
        out[k] = plane.T
    order = {c: j for j, (c, _) in enumerate(chans)}
    assert all(t == 1 for _, t in chans)  # HALF
    return out[..., [order["R"], order["G"], order["B"]]], (x0, y0), disp


def test_exr_half_conversion_and_windows(tmp_path):
    img = _image()
    p = str(tmp_path / "a.EXR")  # suffix test is case-insensitive
    ptgpu.write_image(p, img, full_res=(64, 20), offset=(5, 3))
    got, org, disp = read_exr(p)
    assert org == (5, 3) and disp == (0, 0, 63, 19)
    with np.errstate(over="ignore"):
        ref = img.astype(np.float16)
    assert np.array_equal(got.view(np.uint16), ref.view(np.uint16))
    assert np.isinf(got[0, 1, 0]) and got[0, 1, 2] == 65504


def test_pfm_round_trip(tmp_path):
    img = _image(seed=1)
    p = str(tmp_path / "a.pfm")
    ptgpu.write_image(p, img)
    b = open(p, "rb").read()
    assert b.startswith(b"PF\n37 11\n-1\n")
    data = np.frombuffer(b[len(b"PF\n37 11\n-1\n"):], np.float32).reshape(11, 37, 3)[::-1]
    assert np.array_equal(data, img)


def _bytes_ref(img):
    return np.array([to_byte(v) for v in img.ravel()], np.uint8).reshape(img.shape)


def test_png_pixels(tmp_path):
    img = _image(seed=2)
    p = str(tmp_path / "a.png")
    ptgpu.write_image(p, img)
    b = open(p, "rb").read()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, hdr = 8, b"", None
    while pos < len(b):
        n = struct.unpack(">I", b[pos:pos + 4])[0]
        typ, data = b[pos + 4:pos + 8], b[pos + 8:pos + 8 + n]
        crc = struct.unpack(">I", b[pos + 8 + n:pos + 12 + n])[0]
        assert crc == zlib.crc32(typ + data) & 0xFFFFFFFF
        if typ == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", data)
        elif typ == b"IDAT":
            idat += data
        pos += 12 + n
    assert hdr == (37, 11, 8, 2, 0, 0, 0)
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(11, 1 + 37 * 3)
    assert np.all(raw[:, 0] == 0)
    assert np.array_equal(raw[:, 1:].reshape(11, 37, 3), _bytes_ref(img))


def test_tga_pixels(tmp_path):
    img = _image(seed=3)
    p = str(tmp_path / "a.tga")
    ptgpu.write_image(p, img)
    b = open(p, "rb").read()
    assert b[2] == 2 and struct.unpack("<HH", b[12:16]) == (37, 11) and b[16] == 24 and b[17] == 0x20
    px = np.frombuffer(b[18:18 + 37 * 11 * 3], np.uint8).reshape(11, 37, 3)[..., ::-1]
    assert np.array_equal(px, _bytes_ref(img))
    assert b.endswith(b"TRUEVISION-XFILE.\x00")


def test_unknown_suffix_is_an_error(tmp_path):
    with pytest.raises(ptgpu.PtError) as e:
        ptgpu.write_image(str(tmp_path / "a.jpg"), _image())
    assert e.value.status == 1


def test_film_filename_and_crop(tmp_path):
    from conftest import scene_variant
    p = scene_variant(tmp_path, res=(40, 30), spp=1)
    import re
    txt = open(p).read()
    assert ptgpu.HostScene(p).film_filename == re.search(r'"string filename" \[?"([^"]+)"\]?', txt).group(1)
    q = tmp_path / "d.pbrt"
    q.write_text(re.sub(r'"string filename" \[?"[^"]+"\]?', "", txt))
    assert ptgpu.HostScene(str(q)).film_filename == "pbrt.exr"  # CreateFilm default (film.cpp:225)
    q = tmp_path / "c.pbrt"
    txt = re.sub(r'"string filename" \[?"[^"]+"\]?', "", txt).replace(
        'Film "image"', 'Film "image" "string filename" "out.png" "float cropwindow" [0.25 0.75 0.1 0.5]')
    q.write_text(txt)
    hs = ptgpu.HostScene(str(q))
    assert hs.film_filename == "out.png"
    w, h = hs.film_size()
    assert (w, h) == (20, 12)
    img = _image(w, h, seed=4)
    out = hs.write_image(img, str(tmp_path / "c.exr"))
    got, org, disp = read_exr(out)
    assert org == (10, 3) and disp == (0, 0, 39, 29)
    with np.errstate(over="ignore"):
        assert np.array_equal(got.view(np.uint16), img.astype(np.float16).view(np.uint16))

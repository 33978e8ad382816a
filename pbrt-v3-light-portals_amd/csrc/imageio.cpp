// imageio.cpp -- Film output (Film::WriteImage -> WriteImage, reference
// src/core/imageio.cpp:81-122): the format is chosen by the file suffix
// (case-insensitive HasExtension, src/core/fileutil.cpp):
//   .exr  RGB half-float scanlines, display window = full resolution, data
//         window = the cropped pixel bounds (imageio.cpp:164-187).  Written
//         here without compression (OpenEXR's reader accepts every
//         compression; pixel values, not compressed bytes, are the contract).
//   .pfm  little-endian float RGB, bottom-to-top rows (imageio.cpp WritePFM).
//   .png / .tga  8 bits per channel after GammaCorrect (pbrt.h:298-301) with
//         TO_BYTE = (uint8_t)Clamp(255 * GammaCorrect(v) + 0.5, 0, 255)
//         (imageio.cpp:91-105).  PNG is a plain 24-bit RGB image whose zlib
//         stream uses stored blocks (lodepng's compressed bytes are not part of
//         the contract); TGA is uncompressed BGR, top-to-bottom
//         (imageio.cpp:190-213, ext/targa.cpp tga_write_bgr).
// No third-party image library is used.
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "host_common.h"

namespace pt {

namespace {

bool has_extension(const std::string& name, const char* ext) {
    size_t n = std::strlen(ext);
    if (name.size() < n) return false;
    for (size_t i = 0; i < n; ++i)
        if (std::tolower((unsigned char)name[name.size() - n + i]) != std::tolower((unsigned char)ext[i])) return false;
    return true;
}

struct File {
    FILE* f;
    std::string path;
    explicit File(const std::string& p) : f(std::fopen(p.c_str(), "wb")), path(p) {
        if (!f) throw PtError(PT_ERR_IO, "cannot open \"" + p + "\" for writing");
    }
    ~File() {
        if (f) std::fclose(f);
    }
    void put(const void* d, size_t n) {
        if (n && std::fwrite(d, 1, n, f) != n) throw PtError(PT_ERR_IO, "write error on \"" + path + "\"");
    }
    void close() {
        if (std::fclose(f) != 0) {
            f = nullptr;
            throw PtError(PT_ERR_IO, "write error on \"" + path + "\"");
        }
        f = nullptr;
    }
};

void put_le32(std::vector<uint8_t>& b, uint32_t v) {
    for (int i = 0; i < 4; ++i) b.push_back(uint8_t(v >> (8 * i)));
}
void put_le64(std::vector<uint8_t>& b, uint64_t v) {
    for (int i = 0; i < 8; ++i) b.push_back(uint8_t(v >> (8 * i)));
}
void put_be32(std::vector<uint8_t>& b, uint32_t v) {
    for (int i = 3; i >= 0; --i) b.push_back(uint8_t(v >> (8 * i)));
}
void put_str(std::vector<uint8_t>& b, const char* s) {
    b.insert(b.end(), s, s + std::strlen(s) + 1);
}

}  // namespace

// IEEE binary32 -> binary16, round to nearest even; overflow -> infinity,
// NaN stays NaN (the behaviour of OpenEXR's half(float)).
uint16_t float_to_half(float x) {
    uint32_t u;
    std::memcpy(&u, &x, 4);
    const uint16_t sign = uint16_t((u >> 16) & 0x8000u);
    const uint32_t au = u & 0x7fffffffu;
    if (au >= 0x7f800000u) return uint16_t(sign | 0x7c00u | (au > 0x7f800000u ? 0x200u | ((au >> 13) & 0x3ffu) : 0));
    if (au >= 0x477ff000u) return uint16_t(sign | 0x7c00u);  // rounds to >= 65520 -> inf
    if (au < 0x38800000u) {                                   // half subnormal or zero
        if (au < 0x33000000u) return sign;                    // < 2^-25: rounds to 0
        const uint32_t m = (au & 0x7fffffu) | 0x800000u;
        const int e = int(au >> 23);                          // 102 .. 112
        const int shift = 126 - e;                            // 14 .. 24
        uint32_t h = m >> shift;
        const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) ++h;
        return uint16_t(sign | h);
    }
    uint32_t h = ((au - 0x38000000u) >> 13);  // rebias exponent 127 -> 15
    const uint32_t rem = au & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
    return uint16_t(sign | h);
}

static void write_exr(const std::string& name, const float* rgb, int xres, int yres, int totalX, int totalY, int x0,
                      int y0) {
    std::vector<uint8_t> h = {0x76, 0x2f, 0x31, 0x01, 2, 0, 0, 0};  // magic, version 2 (single-part scanline)
    auto attr = [&](const char* n, const char* type, const std::vector<uint8_t>& v) {
        put_str(h, n);
        put_str(h, type);
        put_le32(h, (uint32_t)v.size());
        h.insert(h.end(), v.begin(), v.end());
    };
    std::vector<uint8_t> ch;
    for (const char* c : {"B", "G", "R"}) {  // channel list is sorted by name
        put_str(ch, c);
        put_le32(ch, 1);  // HALF
        put_le32(ch, 0);  // pLinear + reserved
        put_le32(ch, 1);  // xSampling
        put_le32(ch, 1);  // ySampling
    }
    ch.push_back(0);
    attr("channels", "chlist", ch);
    attr("compression", "compression", {0});  // NO_COMPRESSION
    std::vector<uint8_t> dw, disp;
    put_le32(dw, (uint32_t)x0), put_le32(dw, (uint32_t)y0), put_le32(dw, (uint32_t)(x0 + xres - 1)),
        put_le32(dw, (uint32_t)(y0 + yres - 1));
    put_le32(disp, 0), put_le32(disp, 0), put_le32(disp, (uint32_t)(totalX - 1)), put_le32(disp, (uint32_t)(totalY - 1));
    attr("dataWindow", "box2i", dw);
    attr("displayWindow", "box2i", disp);
    attr("lineOrder", "lineOrder", {0});  // INCREASING_Y
    std::vector<uint8_t> one;
    float onef = 1.f, zero = 0.f;
    uint32_t ub;
    std::memcpy(&ub, &onef, 4);
    put_le32(one, ub);
    attr("pixelAspectRatio", "float", one);
    std::vector<uint8_t> swc;
    std::memcpy(&ub, &zero, 4);
    put_le32(swc, ub), put_le32(swc, ub);
    attr("screenWindowCenter", "v2f", swc);
    attr("screenWindowWidth", "float", one);
    h.push_back(0);  // end of header
    const uint64_t lineBytes = 8 + (uint64_t)xres * 3 * 2;
    const uint64_t first = h.size() + 8ull * (uint64_t)yres;
    for (int y = 0; y < yres; ++y) put_le64(h, first + (uint64_t)y * lineBytes);
    File f(name);
    f.put(h.data(), h.size());
    std::vector<uint8_t> line;
    for (int y = 0; y < yres; ++y) {
        line.clear();
        put_le32(line, (uint32_t)(y0 + y));
        put_le32(line, (uint32_t)(xres * 3 * 2));
        for (int c = 2; c >= 0; --c)  // B, G, R planes
            for (int x = 0; x < xres; ++x) {
                uint16_t v = float_to_half(rgb[3 * ((size_t)y * xres + x) + c]);
                line.push_back(uint8_t(v)), line.push_back(uint8_t(v >> 8));
            }
        f.put(line.data(), line.size());
    }
    f.close();
}

void write_pfm(const std::string& name, const float* rgb, int xres, int yres) {  // imageio.cpp WritePFM
    File f(name);
    char hdr[64];
    int n = std::snprintf(hdr, sizeof hdr, "PF\n%d %d\n-1\n", xres, yres);  // negative scale = little endian
    f.put(hdr, (size_t)n);
    for (int y = yres - 1; y >= 0; --y) f.put(rgb + (size_t)3 * xres * y, sizeof(float) * 3 * (size_t)xres);
    f.close();
}

static float gamma_correct(float v) {  // pbrt.h:298-301
    if (v <= 0.0031308f) return 12.92f * v;
    return 1.055f * std::pow(v, (float)(1.f / 2.4f)) - 0.055f;
}

uint8_t to_byte(float v) {  // imageio.cpp:91 TO_BYTE
    float x = 255.f * gamma_correct(v) + 0.5f;
    x = x < 0.f ? 0.f : (x > 255.f ? 255.f : x);
    return (uint8_t)x;
}

static uint32_t crc32_update(uint32_t c, const uint8_t* p, size_t n) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t k = i;
            for (int j = 0; j < 8; ++j) k = (k & 1) ? 0xedb88320u ^ (k >> 1) : k >> 1;
            table[i] = k;
        }
        init = true;
    }
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return c;
}

static void write_png(const std::string& name, const uint8_t* rgb8, int xres, int yres) {
    std::vector<uint8_t> raw;  // filter byte 0 + row
    raw.reserve((size_t)yres * (1 + 3 * (size_t)xres));
    for (int y = 0; y < yres; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), rgb8 + (size_t)3 * xres * y, rgb8 + (size_t)3 * xres * (y + 1));
    }
    std::vector<uint8_t> z = {0x78, 0x01};  // zlib header, stored deflate blocks
    for (size_t off = 0; off < raw.size() || off == 0;) {
        size_t n = std::min<size_t>(65535, raw.size() - off);
        bool last = off + n == raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back(uint8_t(n)), z.push_back(uint8_t(n >> 8));
        z.push_back(uint8_t(~n)), z.push_back(uint8_t((~n) >> 8));
        z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
        off += n;
        if (last) break;
    }
    uint32_t a = 1, b = 0;  // adler32
    for (uint8_t v : raw) a = (a + v) % 65521u, b = (b + a) % 65521u;
    put_be32(z, (b << 16) | a);
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    auto chunk = [&](const char* type, const std::vector<uint8_t>& data) {
        put_be32(out, (uint32_t)data.size());
        size_t start = out.size();
        out.insert(out.end(), type, type + 4);
        out.insert(out.end(), data.begin(), data.end());
        put_be32(out, crc32_update(0xffffffffu, out.data() + start, out.size() - start) ^ 0xffffffffu);
    };
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, (uint32_t)xres), put_be32(ihdr, (uint32_t)yres);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit, truecolour RGB, deflate, no filter, no interlace
    chunk("IHDR", ihdr);
    chunk("IDAT", z);
    chunk("IEND", {});
    File f(name);
    f.put(out.data(), out.size());
    f.close();
}

static void write_tga(const std::string& name, const uint8_t* rgb8, int xres, int yres) {
    if (xres > 65535 || yres > 65535) throw PtError(PT_ERR_INVALID_ARG, "TGA resolution exceeds 65535");
    std::vector<uint8_t> b = {0, 0, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // no id / colour map; type 2 (BGR); origin 0,0
    b.push_back(uint8_t(xres)), b.push_back(uint8_t(xres >> 8));
    b.push_back(uint8_t(yres)), b.push_back(uint8_t(yres >> 8));
    b.push_back(24);    // pixel depth
    b.push_back(0x20);  // top-to-bottom
    for (size_t i = 0; i < (size_t)xres * yres; ++i)
        b.push_back(rgb8[3 * i + 2]), b.push_back(rgb8[3 * i + 1]), b.push_back(rgb8[3 * i]);
    static const char footer[26] = {0, 0, 0, 0, 0, 0, 0, 0, 'T', 'R', 'U', 'E', 'V', 'I', 'S', 'I', 'O',
                                    'N', '-', 'X', 'F', 'I', 'L', 'E', '.', 0};
    b.insert(b.end(), footer, footer + 26);
    File f(name);
    f.put(b.data(), b.size());
    f.close();
}

void write_image(const std::string& name, const float* rgb, int xres, int yres, int totalX, int totalY, int x0,
                 int y0) {
    if (!rgb || xres <= 0 || yres <= 0) throw PtError(PT_ERR_INVALID_ARG, "write_image: empty image");
    if (has_extension(name, ".exr")) {
        write_exr(name, rgb, xres, yres, totalX, totalY, x0, y0);
    } else if (has_extension(name, ".pfm")) {
        write_pfm(name, rgb, xres, yres);
    } else if (has_extension(name, ".tga") || has_extension(name, ".png")) {
        std::vector<uint8_t> rgb8((size_t)3 * xres * yres);
        for (size_t i = 0; i < rgb8.size(); ++i) rgb8[i] = to_byte(rgb[i]);
        if (has_extension(name, ".tga"))
            write_tga(name, rgb8.data(), xres, yres);
        else
            write_png(name, rgb8.data(), xres, yres);
    } else {
        throw PtError(PT_ERR_INVALID_ARG, "Can't determine image file type from suffix of filename \"" + name + "\"");
    }
}

}  // namespace pt

// spectrum.cpp -- spectral scene parameters: reduction to RGB for the RGB
// build, and the 60-bin SampledSpectrum representation (400-700 nm) the
// hero-wavelength integrators run in (PBRT_SAMPLED_SPECTRUM build,
// spectrum.h:304-440, spectrum.cpp:59-178).
//
// pbrt-v3 is built with Spectrum = RGBSpectrum (`PBRT_SAMPLED_SPECTRUM` off,
// reference src/core/pbrt.h), so every "spectrum" / "blackbody" / "xyz"
// parameter is reduced to RGB when the ParamSet is built
// (src/core/paramset.cpp:122-208) and the renderer only ever sees RGB
// triples.  This file restates that reduction on the host, in the
// reference's float arithmetic order:
//   RGBSpectrum::FromSampled   spectrum.h (class RGBSpectrum) -- projection of
//                              the piecewise-linear SPD onto the 1 nm CIE
//                              x̄ȳz̄ tables, then XYZToRGB (spectrum.h:58-62)
//   InterpolateSpectrumSamples spectrum.cpp:179-188, FindInterval pbrt.h:408-420
//   SortSpectrumSamples        spectrum.cpp:41-57
//   Blackbody(Normalized)      spectrum.cpp:939-964
//   ReadFloatFile              src/core/floatfile.cpp (SPD files)
#include <algorithm>
#include <cctype>
#include <cmath>
#include <limits>
#include <cstdlib>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

#include "host_common.h"
#include "spectral_tables.inc"

namespace pt {

static const int kNCIE = 471;
static const float kInfF = std::numeric_limits<float>::infinity();
static const float kCIE_Y_integral = 106.856895f;  // spectrum.h:83

static float lerpf(float t, float a, float b) { return (1 - t) * a + t * b; }  // pbrt.h:422

float interpolate_spectrum_samples(const float* lambda, const float* vals, int n, float l) {
    for (int i = 0; i < n - 1; ++i)
        if (!(lambda[i + 1] > lambda[i]))
            throw PtError(PT_ERR_PARSE, "spectrum wavelengths must be strictly increasing");
    if (l <= lambda[0]) return vals[0];
    if (l >= lambda[n - 1]) return vals[n - 1];
    // FindInterval: last index whose lambda <= l, clamped to [0, n-2]
    int first = 0, len = n;
    while (len > 0) {
        int half = len >> 1, middle = first + half;
        if (lambda[middle] <= l) {
            first = middle + 1;
            len -= half + 1;
        } else
            len = half;
    }
    int off = std::min(std::max(first - 1, 0), n - 2);
    float t = (l - lambda[off]) / (lambda[off + 1] - lambda[off]);
    return lerpf(t, vals[off], vals[off + 1]);
}

void xyz_to_rgb(const float xyz[3], float rgb[3]) {  // spectrum.h:58-62
    rgb[0] = 3.240479f * xyz[0] - 1.537150f * xyz[1] - 0.498535f * xyz[2];
    rgb[1] = -0.969256f * xyz[0] + 1.875991f * xyz[1] + 0.041556f * xyz[2];
    rgb[2] = 0.055648f * xyz[0] - 0.204043f * xyz[1] + 1.057311f * xyz[2];
}

void rgb_from_sampled(const float* lambda_in, const float* v_in, int n, float rgb[3]) {
    if (n <= 0) throw PtError(PT_ERR_PARSE, "empty spectrum");
    std::vector<float> lambda(lambda_in, lambda_in + n), v(v_in, v_in + n);
    bool sorted = true;
    for (int i = 0; i < n - 1; ++i)
        if (lambda[i] > lambda[i + 1]) sorted = false;
    if (!sorted) {  // SortSpectrumSamples: std::sort of (lambda, value) pairs
        std::vector<std::pair<float, float>> s;
        for (int i = 0; i < n; ++i) s.emplace_back(lambda[i], v[i]);
        std::sort(s.begin(), s.end());
        for (int i = 0; i < n; ++i) lambda[i] = s[i].first, v[i] = s[i].second;
    }
    float xyz[3] = {0, 0, 0};
    for (int i = 0; i < kNCIE; ++i) {
        float val = interpolate_spectrum_samples(lambda.data(), v.data(), n, kCIE_lambda[i]);
        xyz[0] += val * kCIE_X[i];
        xyz[1] += val * kCIE_Y[i];
        xyz[2] += val * kCIE_Z[i];
    }
    const float scale = float(kCIE_lambda[kNCIE - 1] - kCIE_lambda[0]) / float(kCIE_Y_integral * kNCIE);
    xyz[0] *= scale;
    xyz[1] *= scale;
    xyz[2] *= scale;
    xyz_to_rgb(xyz, rgb);
}

void blackbody_radiance(const float* lambda, int n, float T, float* Le) {  // spectrum.cpp:939-955
    if (T <= 0) {
        for (int i = 0; i < n; ++i) Le[i] = 0.f;
        return;
    }
    const float c = (float)299792458;  // int -> float, as the reference compiles it
    const float h = 6.62606957e-34;
    const float kb = 1.3806488e-23;
    for (int i = 0; i < n; ++i) {
        float l = lambda[i] * 1e-9;
        float lambda5 = (l * l) * (l * l) * l;
        Le[i] = (2 * h * c * c) / (lambda5 * (std::exp((h * c) / (l * kb * T)) - 1));
    }
}

void rgb_from_blackbody(float T, float scale, float rgb[3]) {  // paramset.cpp:134-150
    std::vector<float> v(kNCIE);
    blackbody_radiance(kCIE_lambda, kNCIE, T, v.data());
    float lambdaMax = 2.8977721e-3 / T * 1e9;  // BlackbodyNormalized, spectrum.cpp:957-964
    float maxL;
    blackbody_radiance(&lambdaMax, 1, T, &maxL);
    for (int i = 0; i < kNCIE; ++i) v[i] /= maxL;
    float s[3];
    rgb_from_sampled(kCIE_lambda, v.data(), kNCIE, s);
    for (int k = 0; k < 3; ++k) rgb[k] = scale * s[k];
}

// ---------------------------------------------------------------------------
// SampledSpectrum (60 bins over [400, 700] nm)
// ---------------------------------------------------------------------------
// AverageSpectrumSamples (spectrum.cpp:59-90): the segment sums are formed in
// double (`0.5 * (...)` promotes) and narrowed to float on each +=.
float average_spectrum_samples(const float* lambda, const float* vals, int n, float l0, float l1) {
    if (l1 <= lambda[0]) return vals[0];
    if (l0 >= lambda[n - 1]) return vals[n - 1];
    if (n == 1) return vals[0];
    float sum = 0;
    if (l0 < lambda[0]) sum += vals[0] * (lambda[0] - l0);
    if (l1 > lambda[n - 1]) sum += vals[n - 1] * (l1 - lambda[n - 1]);
    int i = 0;
    while (l0 > lambda[i + 1]) ++i;
    auto interp = [&](float w, int k) { return lerpf((w - lambda[k]) / (lambda[k + 1] - lambda[k]), vals[k], vals[k + 1]); };
    for (; i + 1 < n && l1 >= lambda[i]; ++i) {
        const float a = std::max(l0, lambda[i]), b = std::min(l1, lambda[i + 1]);
        sum = (float)((double)sum + 0.5 * (double)(interp(a, i) + interp(b, i)) * (double)(b - a));
    }
    return sum / (l1 - l0);
}

static void bin_range(int i, float* l0, float* l1) {  // Lerp(Float(i) / Float(60), 400, 700)
    *l0 = lerpf(float(i) / float(kNSpec), (float)kLambdaStart, (float)kLambdaEnd);
    *l1 = lerpf(float(i + 1) / float(kNSpec), (float)kLambdaStart, (float)kLambdaEnd);
}

const SpecTables60& spectral_tables() {  // SampledSpectrum::Init (spectrum.h:330-393)
    static SpecTables60 t;
    static bool init = false;
    if (!init) {
        const float* refl[7] = {kRGBRefl2SpectWhite, kRGBRefl2SpectCyan, kRGBRefl2SpectMagenta, kRGBRefl2SpectYellow,
                                kRGBRefl2SpectRed, kRGBRefl2SpectGreen, kRGBRefl2SpectBlue};
        const float* illum[7] = {kRGBIllum2SpectWhite, kRGBIllum2SpectCyan, kRGBIllum2SpectMagenta,
                                 kRGBIllum2SpectYellow, kRGBIllum2SpectRed, kRGBIllum2SpectGreen, kRGBIllum2SpectBlue};
        for (int i = 0; i < kNSpec; ++i) {
            float l0, l1;
            bin_range(i, &l0, &l1);
            t.X[i] = average_spectrum_samples(kCIE_lambda, kCIE_X, kNCIE, l0, l1);
            t.Y[i] = average_spectrum_samples(kCIE_lambda, kCIE_Y, kNCIE, l0, l1);
            t.Z[i] = average_spectrum_samples(kCIE_lambda, kCIE_Z, kNCIE, l0, l1);
            for (int k = 0; k < 7; ++k) {
                t.refl[k][i] = average_spectrum_samples(kRGB2SpectLambda, refl[k], 32, l0, l1);
                t.illum[k][i] = average_spectrum_samples(kRGB2SpectLambda, illum[k], 32, l0, l1);
            }
        }
        init = true;
    }
    return t;
}

void s60_from_sampled(const float* lambda_in, const float* v_in, int n, float out[60]) {  // spectrum.h:310-328
    if (n <= 0) throw PtError(PT_ERR_PARSE, "empty spectrum");
    std::vector<float> lambda(lambda_in, lambda_in + n), v(v_in, v_in + n);
    bool sorted = true;
    for (int i = 0; i < n - 1; ++i)
        if (lambda[i] > lambda[i + 1]) sorted = false;
    if (!sorted) {
        std::vector<std::pair<float, float>> sv;
        for (int i = 0; i < n; ++i) sv.emplace_back(lambda[i], v[i]);
        std::sort(sv.begin(), sv.end());
        for (int i = 0; i < n; ++i) lambda[i] = sv[i].first, v[i] = sv[i].second;
    }
    for (int i = 0; i < n - 1; ++i)
        if (!(lambda[i + 1] > lambda[i]))
            throw PtError(PT_ERR_PARSE, "spectrum wavelengths must be strictly increasing");
    for (int i = 0; i < kNSpec; ++i) {
        float l0, l1;
        bin_range(i, &l0, &l1);
        out[i] = average_spectrum_samples(lambda.data(), v.data(), n, l0, l1);
    }
}

// SampledSpectrum::FromRGB (spectrum.cpp:98-172): Smits' basis, then Clamp().
void s60_from_rgb(const float rgb[3], bool reflectance, float out[60]) {
    const SpecTables60& t = spectral_tables();
    const float(*b)[60] = reflectance ? t.refl : t.illum;  // W C M Y R G B
    enum { W, C, M, Y, R, G, B };
    float r[60] = {0};
    auto add = [&](float a, int k) { for (int i = 0; i < kNSpec; ++i) r[i] += b[k][i] * a; };
    if (rgb[0] <= rgb[1] && rgb[0] <= rgb[2]) {
        add(rgb[0], W);
        if (rgb[1] <= rgb[2]) { add(rgb[1] - rgb[0], C); add(rgb[2] - rgb[1], B); }
        else { add(rgb[2] - rgb[0], C); add(rgb[1] - rgb[2], G); }
    } else if (rgb[1] <= rgb[0] && rgb[1] <= rgb[2]) {
        add(rgb[1], W);
        if (rgb[0] <= rgb[2]) { add(rgb[0] - rgb[1], M); add(rgb[2] - rgb[0], B); }
        else { add(rgb[2] - rgb[1], M); add(rgb[0] - rgb[2], R); }
    } else {
        add(rgb[2], W);
        if (rgb[0] <= rgb[1]) { add(rgb[0] - rgb[2], Y); add(rgb[1] - rgb[0], G); }
        else { add(rgb[1] - rgb[2], Y); add(rgb[0] - rgb[1], R); }
    }
    const float sc = reflectance ? (float).94 : .86445f;
    for (int i = 0; i < kNSpec; ++i) {
        r[i] *= sc;
        out[i] = r[i] < 0 ? 0.f : (r[i] > kInfF ? kInfF : r[i]);  // Clamp(0, Infinity)
    }
}

void s60_to_xyz(const float s[60], float xyz[3]) {  // SampledSpectrum::ToXYZ (spectrum.h:395-406)
    const SpecTables60& t = spectral_tables();
    xyz[0] = xyz[1] = xyz[2] = 0.f;
    for (int i = 0; i < kNSpec; ++i) {
        xyz[0] += t.X[i] * s[i];
        xyz[1] += t.Y[i] * s[i];
        xyz[2] += t.Z[i] * s[i];
    }
    const float scale = float(kLambdaEnd - kLambdaStart) / float(kCIE_Y_integral * kNSpec);
    xyz[0] *= scale;
    xyz[1] *= scale;
    xyz[2] *= scale;
}

float s60_y(const float s[60]) {  // SampledSpectrum::y (spectrum.h:407-413)
    const SpecTables60& t = spectral_tables();
    float yy = 0.f;
    for (int i = 0; i < kNSpec; ++i) yy += t.Y[i] * s[i];
    return yy * float(kLambdaEnd - kLambdaStart) / float(kCIE_Y_integral * kNSpec);
}

void s60_blackbody(float T, float scale, float out[60]) {  // paramset.cpp:134-150, SampledSpectrum build
    std::vector<float> v(kNCIE);
    blackbody_radiance(kCIE_lambda, kNCIE, T, v.data());
    float lambdaMax = 2.8977721e-3 / T * 1e9;
    float maxL;
    blackbody_radiance(&lambdaMax, 1, T, &maxL);
    for (int i = 0; i < kNCIE; ++i) v[i] /= maxL;
    s60_from_sampled(kCIE_lambda, v.data(), kNCIE, out);
    for (int i = 0; i < kNSpec; ++i) out[i] = out[i] * scale;
}

void copper_spectrum(bool k, float rgb[3]) {  // metal.cpp:116-122
    rgb_from_sampled(kCopperWavelengths, k ? kCopperK : kCopperN, 56, rgb);
}

// ReadFloatFile (floatfile.cpp:40-86): a character state machine -- numbers
// are runs of [0-9.e+-] started by [0-9.+-], '#' comments to end of line, a
// number still open at EOF is dropped.  Returns false when the file cannot
// be opened (the caller then uses a black spectrum, paramset.cpp:183-188).
bool read_float_file(const std::string& path, std::vector<float>* values) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return false;
    int c;
    bool inNumber = false;
    char cur[32];
    int pos = 0;
    while ((c = std::getc(f)) != EOF) {
        if (inNumber) {
            if (pos >= (int)sizeof cur) {
                std::fclose(f);
                throw PtError(PT_ERR_PARSE, "overflowed number buffer in float file \"" + path + "\"");
            }
            if (std::isdigit(c) || c == '.' || c == 'e' || c == '-' || c == '+')
                cur[pos++] = (char)c;
            else {
                cur[pos++] = '\0';
                values->push_back((float)std::atof(cur));
                inNumber = false;
                pos = 0;
            }
        } else if (std::isdigit(c) || c == '.' || c == '-' || c == '+') {
            inNumber = true;
            cur[pos++] = (char)c;
        } else if (c == '#') {
            while ((c = std::getc(f)) != '\n' && c != EOF) {
            }
        }
    }
    std::fclose(f);
    return true;
}

}  // namespace pt

#!/usr/bin/env python3
"""The INTEGRATION.md §1 accessor patch, applied to a pbrt-v3-light-portals
source tree (a COPY: the test copies the reference's headers to a temporary
directory first; nothing is written under the reference).

Each edit inserts one-line read accessors into a class of the reference's
headers -- the members the reference keeps private that GpuPathIntegrator
(integration/gpupath.cpp) reads.  The patch edits headers only and adds no
state a .cpp file would have to set: the binding reads the BVH through
BVHAccel::nodes (a pointer to the still-incomplete LinearBVHNode of bvh.h:52,
whose 32-byte layout bvh.cpp:95-104 the binding mirrors and counts by walking
the tree from node 0), and the constant radiance of an InfiniteAreaLight from
its own Lmap (the 1x1 MIPMap infinite.cpp:43-61 builds).  The one member it
adds, Sphere::phiMaxDegrees, is set in the constructor's init list, which
sphere.h holds.
The same getters appear, marked PATCH, in the stub mirror
integration/pbrt_stub/stub_pbrt.h; tests/test_gpupath_reference_headers.py
checks that the two name the same accessors.

Edits are anchored on the class head ("class X : public Y {") and its first
"public:" / "private:" / "protected:" label, not on line numbers, so the patch
states what is added rather than restating the reference's text.

usage: accessor_patch.py <copy of reference src/>
"""
import os
import re
import sys

# (header, class, getters inserted after the class's first "public:",
#  members inserted before the class's closing "};" (own access label), ctor init-list edits (old, new))
PATCH = [
    ("core/scene.h", "Scene", [
        "const Primitive *GetAggregate() const { return aggregate.get(); }",
    ], [], []),
    ("accelerators/bvh.h", "BVHAccel", [
        "const std::vector<std::shared_ptr<Primitive>> &GetPrimitives() const { return primitives; }",
        "const LinearBVHNode *GetNodes() const { return nodes; }",
    ], [], []),
    ("core/primitive.h", "GeometricPrimitive", [
        "const Shape *GetShape() const { return shape.get(); }",
    ], [], []),
    ("shapes/triangle.h", "Triangle", [
        "const TriangleMesh *GetMesh() const { return mesh.get(); }",
        "const int *GetVertexIndices() const { return v; }",
    ], [], []),
    ("lights/diffuse.h", "DiffuseAreaLight", [
        "const Spectrum &GetLemit() const { return Lemit; }",
        "bool TwoSided() const { return twoSided; }",
        "const Shape *GetShape() const { return shape.get(); }",
    ], [], []),
    ("materials/matte.h", "MatteMaterial", [
        "const std::shared_ptr<Texture<Spectrum>> &GetKd() const { return Kd; }",
        "const std::shared_ptr<Texture<Float>> &GetSigma() const { return sigma; }",
    ], [], []),
    ("materials/metal.h", "MetalMaterial", [
        "const std::shared_ptr<Texture<Spectrum>> &GetEta() const { return eta; }",
        "const std::shared_ptr<Texture<Spectrum>> &GetK() const { return k; }",
        "const std::shared_ptr<Texture<Float>> &GetRoughness() const { return roughness; }",
        "const std::shared_ptr<Texture<Float>> &GetURoughness() const { return uRoughness; }",
        "const std::shared_ptr<Texture<Float>> &GetVRoughness() const { return vRoughness; }",
        "bool RemapRoughness() const { return remapRoughness; }",
    ], [], []),
    ("materials/glass.h", "GlassMaterial", [
        "const std::shared_ptr<Texture<Spectrum>> &GetKr() const { return Kr; }",
        "const std::shared_ptr<Texture<Spectrum>> &GetKt() const { return Kt; }",
        "const std::shared_ptr<Texture<Float>> &GetURoughness() const { return uRoughness; }",
        "const std::shared_ptr<Texture<Float>> &GetVRoughness() const { return vRoughness; }",
        "const std::shared_ptr<Texture<Float>> &GetIndex() const { return index; }",
        "bool RemapRoughness() const { return remapRoughness; }",
    ], [], []),
    ("materials/dispersive_glass.h", "DispersiveGlassMaterial", [
        "const std::shared_ptr<Texture<Spectrum>> &GetKr() const { return Kr; }",
        "const std::shared_ptr<Texture<Spectrum>> &GetKt() const { return Kt; }",
        "const std::shared_ptr<Texture<Float>> &GetURoughness() const { return uRoughness; }",
        "const std::shared_ptr<Texture<Float>> &GetVRoughness() const { return vRoughness; }",
        "const std::shared_ptr<Texture<Float>> &GetIndexMin() const { return indexMin; }",
        "const std::shared_ptr<Texture<Float>> &GetIndexMax() const { return indexMax; }",
        "bool RemapRoughness() const { return remapRoughness; }",
    ], [], []),
    ("materials/mirror.h", "MirrorMaterial", [
        "const std::shared_ptr<Texture<Spectrum>> &GetKr() const { return Kr; }",
    ], [], []),
    ("materials/plastic.h", "PlasticMaterial", [
        "const std::shared_ptr<Texture<Spectrum>> &GetKd() const { return Kd; }",
        "const std::shared_ptr<Texture<Spectrum>> &GetKs() const { return Ks; }",
        "const std::shared_ptr<Texture<Float>> &GetRoughness() const { return roughness; }",
        "bool RemapRoughness() const { return remapRoughness; }",
    ], [], []),
    ("shapes/sphere.h", "Sphere", [
        "Float Radius() const { return radius; }",
        "Float ZMin() const { return zMin; }",
        "Float ZMax() const { return zMax; }",
        "Float PhiMaxDegrees() const { return phiMaxDegrees; }",
    ], ["Float phiMaxDegrees;  // the creation argument: Radians(Clamp(phiMax, 0, 360)) does not round-trip"],
        [("phiMax(Radians(Clamp(phiMax, 0, 360)))", "phiMax(Radians(Clamp(phiMax, 0, 360))), phiMaxDegrees(phiMax)")]),
    ("lights/point.h", "PointLight", [
        "const Point3f &GetPosition() const { return pLight; }",
        "const Spectrum &GetIntensity() const { return I; }",
    ], [], []),
    ("lights/infinite.h", "InfiniteAreaLight", [
        "const Transform &GetLightToWorld() const { return LightToWorld; }",
        "const MIPMap<RGBSpectrum> *GetLmap() const { return Lmap.get(); }",
    ], [], []),
]

def getter_names(patch=PATCH):
    """{class: sorted accessor names} of the patch."""
    out = {}
    for _, cls, getters, _, _ in patch:
        out[cls] = sorted(re.search(r"(\w+)\(\) const", g).group(1) for g in getters)
    return out


def _class_span(text, cls):
    m = re.search(r"\bclass\s+%s\b[^;{]*\{" % re.escape(cls), text)
    if not m:
        raise ValueError("class %s not found" % cls)
    depth, i = 1, m.end()
    while depth:
        c = text[i]
        depth += (c == "{") - (c == "}")
        i += 1
    return m.start(), m.end(), i - 1  # head start, body start, index of the closing brace


def apply(src_root):
    for rel, cls, getters, members, inits in PATCH:
        path = os.path.join(src_root, rel)
        text = open(path).read()
        for old, new in inits:
            if old not in text:
                raise ValueError("%s: init list %r not found" % (rel, old))
            text = text.replace(old, new, 1)
        _, body, close = _class_span(text, cls)
        if members:
            add = "\n  private:  // PATCH\n" + "".join("    %s\n" % m for m in members)
            text = text[:close] + add + text[close:]
        lab = re.compile(r"\bpublic:").search(text, body)
        if not lab or lab.start() > close:
            raise ValueError("%s: %s has no public: label" % (rel, cls))
        ins = "".join("\n    %s  // PATCH" % g for g in getters)
        text = text[:lab.end()] + ins + text[lab.end():]
        open(path, "w").write(text)


if __name__ == "__main__":
    apply(sys.argv[1])

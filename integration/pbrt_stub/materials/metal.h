// Stub of the reference header src/materials/metal.h for compile/ABI tests of the
// GpuPathIntegrator binding: everything lives in stub_pbrt.h.
#pragma once
#include "stub_pbrt.h"

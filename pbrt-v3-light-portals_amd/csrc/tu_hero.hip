// tu_hero.hip -- translation unit of the hero-wavelength kernels (hero.hip).
#define PT_TU_HERO 1
#include "hero.hip"

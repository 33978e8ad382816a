// tu_misc.hip -- translation unit of the camera, film and debug kernels (kernels.hip).
#define PT_TU_MISC 1
#include "kernels.hip"

// ptrender.cpp -- pbrt-style command line (src/main/pbrt.cpp:43-173 subset)
// on top of the C ABI: ptrender [--outfile f] [--device N | --devices a,b,..] [--quiet]
// [--stats] scene.pbrt.  The image goes to the Film's "filename" (default
// pbrt.exr) unless --outfile overrides it (film.cpp:213-225); the suffix
// picks EXR / PFM / PNG / TGA (Film::WriteImage -> WriteImage, imageio.cpp:81-122).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pt.h"

static void usage() {
    std::fprintf(stderr, "usage: ptrender [--outfile file.{exr,pfm,png,tga}] [--device N | --devices a,b,...] [--quiet] [--stats] scene.pbrt\n");
    std::exit(1);
}

int main(int argc, char** argv) {
    std::string out, scene;
    std::vector<int32_t> devices{0};
    bool quiet = false, stats = false;
    for (int i = 1; i < argc; ++i) {
        if (!std::strcmp(argv[i], "--outfile") && i + 1 < argc) out = argv[++i];
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) devices = {std::atoi(argv[++i])};
        else if (!std::strcmp(argv[i], "--devices") && i + 1 < argc) {  // one process, tiles over these GPUs
            devices.clear();
            for (const char* p = argv[++i]; *p;) {
                devices.push_back((int32_t)std::strtol(p, (char**)&p, 10));
                if (*p == ',') ++p;
                else if (*p) usage();
            }
            if (devices.empty()) usage();
        }
        else if (!std::strcmp(argv[i], "--quiet")) quiet = true;
        else if (!std::strcmp(argv[i], "--stats")) stats = true;
        else if (argv[i][0] == '-') usage();
        else scene = argv[i];
    }
    if (scene.empty()) usage();
    pt_host_scene* hs = nullptr;
    if (pt_load_pbrt(scene.c_str(), &hs) != PT_OK) {
        std::fprintf(stderr, "ptrender: %s\n", pt_last_error());
        return 1;
    }
    if (pt_init((int)devices.size(), devices.data()) != PT_OK) {
        std::fprintf(stderr, "ptrender: %s\n", pt_last_error());
        return 1;
    }
    pt_scene* s = nullptr;
    if (pt_scene_create(pt_host_scene_desc(hs), &s) != PT_OK) {
        std::fprintf(stderr, "ptrender: %s\n", pt_last_error());
        return 1;
    }
    int32_t w = 0, h = 0;
    pt_film_size(s, &w, &h);
    std::vector<float> rgb((size_t)3 * w * h);
    pt_stats st{};
    if (pt_render(s, rgb.data(), &st) != PT_OK) {
        std::fprintf(stderr, "ptrender: %s\n", pt_last_error());
        return 1;
    }
    if (out.empty()) out = pt_host_scene_film_filename(hs);
    if (pt_write_film_image(pt_host_scene_desc(hs), out.c_str(), rgb.data()) != PT_OK) {
        std::fprintf(stderr, "ptrender: %s\n", pt_last_error());
        return 1;
    }
    if (!quiet)
        std::printf("ptrender: %s -> %s (%dx%d), %.1f ms, %.2f Msamples/s\n", scene.c_str(), out.c_str(), w, h,
                    st.render_ms, st.samples / (st.render_ms * 1e3));
    if (stats)
        std::printf("  camera rays %llu  regular ray tests %llu  shadow ray tests %llu  nodes %llu  prims %llu\n",
                    (unsigned long long)st.camera_rays, (unsigned long long)st.closest_rays,
                    (unsigned long long)st.shadow_rays, (unsigned long long)st.node_visits,
                    (unsigned long long)st.prim_tests);
    pt_scene_destroy(s);
    pt_host_scene_free(hs);
    return 0;
}

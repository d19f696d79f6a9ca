// cli.cpp — `raytracing`, the reference's command-line surface (main.cu:29-131) on the MI355X path.
//
//   raytracing [scene] [sN|bN] [sN|bN] [wN] [hN] [gN]
//
// argv[1] selects a catalog scene (main.cu:52-117, plus 20 = random 10k spheres); 'sN' sets samples per
// pixel, 'bN' max bounces (main.cu:118-129).  Additive flags: 'wN'/'hN' override the resolution (the
// reference derives H = (int)(W / ratio), raytracing.cu:1659-1660); 'gN' renders on the first N visible
// devices (rows interleaved, one RCCL gather: rt_render_devices).  Without 'gN' the device is HIP's current
// one (select with HIP_VISIBLE_DEVICES).
// Writes settings.img_name as binary P6 PPM into the current directory, like render() (:1772).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "rt_host.h"
#include "rt_render.h"

int main(int argc, char **argv) {
  const auto t_start = std::chrono::steady_clock::now();   // end-to-end: scene build .. PPM written
  int scene = 0;
  if (argc > 1) scene = std::atoi(argv[1]);
  rt_world *w = rt_world_create(scene == RT_SCENE_RANDOM_10K ? 24000 : 8000, 10u << 20);
  rt_settings s;
  int st = rt_world_build_scene(w, scene, &s);
  if (st == RT_ERR_INVALID_ARG) {
    std::printf("Unknown scene\n");
    rt_world_destroy(w);
    return 1;
  }
  int32_t width = 0, height = 0, gpus = 0;
  for (int a = 2; a < argc; ++a) {
    const char *v = argv[a] + 1;
    switch (argv[a][0]) {
      case 'b': s.max_bounces = std::atoi(v); break;
      case 's': s.samples_per_pixel = std::atoi(v); break;
      case 'w': width = std::atoi(v); break;
      case 'h': height = std::atoi(v); break;
      case 'g': gpus = std::atoi(v); break;
      default: break;
    }
  }
  uint16_t root = 0;
  rt_scene sc;
  if (st != RT_OK || rt_world_build_bvh(w, &root) != RT_OK || rt_world_scene(w, root, &sc) != RT_OK) {
    std::fprintf(stderr, "scene build failed\n");
    rt_world_destroy(w);
    return 1;
  }
  rt_camera cam;
  int32_t W = 0, H = 0;
  if (width > 0 && height <= 0) height = static_cast<int32_t>(width / s.img_ratio);
  if (rt_camera_from_settings(&s, width, height, &cam, &W, &H) != RT_OK) {
    std::fprintf(stderr, "bad camera/resolution\n");
    rt_world_destroy(w);
    return 1;
  }
  rt_params p = {};
  p.width = W; p.height = H; p.row_offset = 0; p.row_stride = 1; p.row_count = H;
  p.samples_per_pixel = s.samples_per_pixel; p.max_bounces = s.max_bounces;
  p.background = s.background; p.seed = 1234; p.flags = 0;
  std::vector<float> fb(static_cast<size_t>(W) * H * 3);
  rt_stats stats;
  if (gpus > 0) {   // one process, N devices (rt_multi.cpp): the float rows are gathered for pixels_to_ppm
    std::vector<int> devs(gpus);
    for (int g = 0; g < gpus; ++g) devs[g] = g;
    st = rt_render_devices(&sc, &cam, &p, devs.data(), gpus, fb.data(), nullptr, &stats);
  } else {
    st = rt_render(&sc, &cam, &p, fb.data(), &stats);
  }
  std::printf("rt_render status: %s\n", rt_status_string(st));
  if (st != RT_OK) {
    rt_world_destroy(w);
    return 2;
  }
  std::printf("Rendering time: %fms\n", stats.render_ms);
  std::printf("Rendering time: %fs\n", stats.render_ms / 1e3);
  std::printf("RNG seeding time: %fms, end-to-end: %fms, %.1f Msamples/s\n", stats.init_ms, stats.total_ms,
              static_cast<double>(stats.samples) / (stats.render_ms * 1e3));
  if (gpus > 0) std::printf("Devices: %d, RCCL gather + un-permute: %fms\n", stats.devices, stats.gather_ms);
  if (rt_write_ppm(s.img_name, fb.data(), static_cast<uint32_t>(W), static_cast<uint32_t>(H)) != RT_OK)
    std::fprintf(stderr, "Couldn't open the file for writing\n");
  const double e2e = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
  static const char *jit_names[] = {"none", "in-process", "disk cache", "compiled"};
  // the reference's render() region (raytracing.cu:1649-1773) plus the scene build before it
  std::printf("End-to-end: %fms (scene + BVH + kernels [%s, %.1f ms] + upload + seed + render + D2H + PPM), "
              "rt_render %fms\n", e2e, jit_names[stats.jit_source & 3], stats.jit_ms, stats.total_ms);
  rt_world_destroy(w);
  return 0;
}

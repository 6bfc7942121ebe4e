// adapter_harness.cpp — TEST HARNESS for the INTEGRATION.md adapter (see
// tests/test_integration_doc.py).  Sets a PathTracer up exactly as the
// reference does (oracle/ref/ref_driver.cpp's restatement of main.cpp +
// Application::load, linked from oracle/_ref objects), then drives the
// adapter the way the reference's call sites would: init(), begin_frame(seed)
// from start_raytracing, raytrace_tile() from 4 worker threads drawing tiles
// from a shared FIFO, and a cancelled frame.  The ABI underneath is the
// capture double (capture_abi.cpp).
// usage: adapter_harness scene.dae W H [envmap.exr|-] [cam.info|-]
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>

#include "gpu_pathtracer.h"

using namespace CMU462;

PathTracer* ref_setup_pathtracer(const char* scene, size_t w, size_t h, size_t spp, size_t depth, size_t lights,
                                 const char* cam, const char* envmap, HDRImageBuffer** env_out);

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const size_t W = std::strtoul(argv[2], nullptr, 10), H = std::strtoul(argv[3], nullptr, 10);
  const char* env = argc > 4 && std::string(argv[4]) != "-" ? argv[4] : nullptr;
  const char* cam = argc > 5 && std::string(argv[5]) != "-" ? argv[5] : nullptr;
  HDRImageBuffer* envmap = nullptr;
  PathTracer* pt = ref_setup_pathtracer(argv[1], W, H, 4, 4, 1, cam, env, &envmap);
  GpuPathTracer gpu(pt, envmap);
  gpu.init();
  // frame 1: start_raytracing's state, one seed, tiles from a shared FIFO on 4 threads
  pt->continueRaytracing = true;
  pt->sampleBuffer.clear();
  pt->frameBuffer.clear();
  gpu.begin_frame(1234u);
  const int ntx = (int)((W + 31) / 32), nt = ntx * (int)((H + 31) / 32);
  std::atomic<int> next(0);
  std::thread th[4];
  for (auto& t : th)
    t = std::thread([&] {
      for (int i; (i = next++) < nt;) gpu.raytrace_tile((i % ntx) * 32, (i / ntx) * 32, 32, 32);
    });
  for (auto& t : th) t.join();
  gpu.finish_tiles();  // the last worker's call site (worker_thread, workerDoneCount == numWorkerThreads)
  // frame 2 (seed 99) cancelled before its tiles: nothing may be launched
  gpu.begin_frame(99u);
  pt->continueRaytracing = false;
  gpu.raytrace_tile(0, 0, 32, 32);
  std::printf("{\"tiles\": %d}\n", nt);
  return 0;
}

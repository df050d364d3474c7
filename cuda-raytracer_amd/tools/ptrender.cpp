// ptrender -- headless replacement of the reference's scottyCuda driver
// (src/cudaMain.cpp:30-104 + display.cpp's GLUT loop): load a COLLADA scene,
// render W x H at S spp on one GPU through the C ABI, write a PFM.  With -v,
// the progressive viewer loop instead (scotty::Viewer): one displayed frame of
// S samples per character of the key script (w/a/s/d move the camera, p
// pauses, '.' no key), ms per frame printed, the last frame written.  With
// -D 0,1,... the frame is split over those GPUs of this process
// (scotty::MultiGpuPathTracer over pt_group: RCCL gather into the first).
//
//   ptrender scene.dae [-w 1024] [-h 1024] [-s 256] [-m 8] [-o out.png|out.pfm] [-d device] [-v keys]
//            [-D devices]
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <iostream>

#include "../scotty/scotty_pt.h"

int main(int argc, char** argv) {
  if (argc < 2) {
    std::cerr << "usage: ptrender scene.dae [-w W] [-h H] [-s spp] [-m bounces] [-o out.png|out.pfm] [-d device] "
                 "[-v viewer-keys]\n";
    return 2;
  }
  int w = 512, h = 512, spp = 16, bounces = 8, dev = 0;
  std::string out = "out.pfm", keys, devlist;
  for (int i = 2; i + 1 < argc; i += 2) {
    std::string k = argv[i];
    if (k == "-w") w = atoi(argv[i + 1]);
    else if (k == "-h") h = atoi(argv[i + 1]);
    else if (k == "-s") spp = atoi(argv[i + 1]);
    else if (k == "-m") bounces = atoi(argv[i + 1]);
    else if (k == "-o") out = argv[i + 1];
    else if (k == "-d") dev = atoi(argv[i + 1]);
    else if (k == "-v") keys = argv[i + 1];
    else if (k == "-D") devlist = argv[i + 1];
  }
  if (!devlist.empty()) {
    std::vector<int> devs;
    for (size_t p = 0; p <= devlist.size();) {
      size_t q = devlist.find(',', p);
      if (q == std::string::npos) q = devlist.size();
      devs.push_back(atoi(devlist.substr(p, q - p).c_str()));
      p = q + 1;
    }
    try {
      scotty::MultiGpuPathTracer pt(devs, spp, bounces);
      pt.set_frame_size(w, h);
      pt.set_scene(std::string(argv[1]));
      auto t0 = std::chrono::steady_clock::now();
      pt.start_raytracing();
      pt.is_done();
      double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      double gms = 0;
      pt_group_timing(pt.group(), &gms, nullptr);
      std::cout << w << "x" << h << " " << spp << " spp " << bounces << " bounces on " << devs.size()
                << " GPUs (" << (pt.gather_kind() == PT_GATHER_RCCL ? "RCCL" : "host") << " gather " << gms
                << " ms): " << s * 1e3 << " ms\n";
      pt.save_image(out);
    } catch (const std::exception& e) {
      std::cerr << "ptrender: " << e.what() << "\n";
      return 1;
    }
    return 0;
  }
  if (!keys.empty()) {
    try {
      scotty::CudaRenderer r(dev);
      r.allocOutputImage(w, h);
      r.loadScene(std::string(argv[1]));
      r.setup();
      scotty::Viewer v(r, spp, bounces);
      const scotty::Image* img = nullptr;
      for (char c : keys) {
        if (c != '.') v.handleKeyPress(c);
        auto t0 = std::chrono::steady_clock::now();
        img = v.renderPicture();
        double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        int n = 0;
        pt_samples(r.device().get(), &n);
        std::cout << "frame " << v.frames() << " key '" << c << "': " << ms << " ms, " << n << " samples\n";
      }
      const bool pfm = out.size() >= 4 && out.compare(out.size() - 4, 4, ".pfm") == 0;
      int rc = pfm ? pt_write_pfm(out.c_str(), img->data.data(), w, h) : 0;
      if (!pfm) {
        std::vector<uint8_t> rgba8((size_t)w * h * 4);
        rc = pt_tonemap(img->data.data(), w, h, 2.2f, 1.0f, rgba8.data());
        if (!rc) rc = pt_write_png(out.c_str(), rgba8.data(), w, h);
      }
      if (rc) throw scotty::Error(rc, "cannot write " + out);
    } catch (const std::exception& e) {
      std::cerr << "ptrender: " << e.what() << "\n";
      return 1;
    }
    return 0;
  }
  try {
    scotty::PathTracer pt(spp, bounces);
    pt.renderer();  // device context created here
    pt.set_frame_size(w, h);
    pt.set_scene(argv[1]);
    auto t0 = std::chrono::steady_clock::now();
    pt.start_raytracing();
    pt.is_done();
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    pt_stats st{};
    pt_get_stats(pt.renderer().device().get(), &st);
    std::cout << w << "x" << h << " " << spp << " spp " << bounces << " bounces: " << s * 1e3 << " ms, "
              << st.rays / s / 1e6 << " Mrays/s\n";
    pt.save_image(out);
    (void)dev;
  } catch (const std::exception& e) {
    std::cerr << "ptrender: " << e.what() << "\n";
    return 1;
  }
  return 0;
}

// iS3D_amd -- drop-in replacement of the reference executable (src/cpp/Main.cpp) for
// operations 1 (continuous spectra) and 0 (spacetime distributions): run in a directory laid out
// like the reference's (iS3D_parameters.dat,
// input/surface.dat, PDG/, deltaf_coefficients/, tables/, results/continuous/).
// Environment: IS3D_DEVICE (first GPU, default 0), IS3D_NUM_GPUS (cells sharded, default 1), or
// IS3D_DEVICES (comma-separated device per cell shard, e.g. "0,1,2,3"; takes precedence).
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <sstream>
#include <string>

#include "is3d_driver.h"

// a non-negative decimal integer, or -1 (malformed: "x", "1x", "-2", "")
static long parse_index(const std::string& s) {
  if (s.empty()) return -1;
  char* end = nullptr;
  errno = 0;
  const long v = std::strtol(s.c_str(), &end, 10);
  if (errno || *end != '\0' || v < 0 || v > 1 << 20) return -1;
  return v;
}

int main(int argc, char** argv) {
  is3d::host::RunOptions opt;
  const int kErrArg = 1;   // IS3D_ERR_ARG
  if (const char* d = std::getenv("IS3D_DEVICE")) {
    const long v = parse_index(d);
    if (v < 0) { std::fprintf(stderr, "iS3D_amd: bad IS3D_DEVICE '%s'\n", d); return kErrArg; }
    opt.device = (int)v;
  }
  if (const char* n = std::getenv("IS3D_NUM_GPUS")) {
    const long v = parse_index(n);
    if (v < 1) { std::fprintf(stderr, "iS3D_amd: bad IS3D_NUM_GPUS '%s'\n", n); return kErrArg; }
    opt.num_devices = (int)v;
  }
  if (const char* l = std::getenv("IS3D_DEVICES")) {
    std::stringstream ss(l);
    std::string tok;
    while (std::getline(ss, tok, ',')) {
      const long v = parse_index(tok);
      if (v < 0) { std::fprintf(stderr, "iS3D_amd: bad device '%s' in IS3D_DEVICES '%s'\n", tok.c_str(), l); return kErrArg; }
      opt.devices.push_back((int)v);
    }
  }
  try {
    is3d::host::IS3D particlization(argc > 1 ? argv[1] : ".");
    particlization.run_particlization(1, opt);
  } catch (const is3d::host::EngineError& e) {
    std::fprintf(stderr, "iS3D_amd: %s\n", e.what());
    return e.code;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "iS3D_amd: %s\n", e.what());
    return 1;
  }
  return 0;
}

// iS3D_amd -- drop-in replacement of the reference executable (src/cpp/Main.cpp) for
// operations 1 (continuous spectra) and 0 (spacetime distributions): run in a directory laid out
// like the reference's (iS3D_parameters.dat,
// input/surface.dat, PDG/, deltaf_coefficients/, tables/, results/continuous/).
// Environment: IS3D_DEVICE (first GPU, default 0), IS3D_NUM_GPUS (cells sharded, default 1), or
// IS3D_DEVICES (comma-separated device per cell shard, e.g. "0,1,2,3"; takes precedence).
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <sstream>
#include <string>

#include "is3d_driver.h"

int main(int argc, char** argv) {
  is3d::host::RunOptions opt;
  if (const char* d = std::getenv("IS3D_DEVICE")) opt.device = std::atoi(d);
  if (const char* n = std::getenv("IS3D_NUM_GPUS")) opt.num_devices = std::atoi(n);
  if (const char* l = std::getenv("IS3D_DEVICES")) {
    std::stringstream ss(l);
    std::string tok;
    while (std::getline(ss, tok, ',')) if (!tok.empty()) opt.devices.push_back(std::atoi(tok.c_str()));
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

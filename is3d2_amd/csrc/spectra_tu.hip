// spectra_tu.hip -- k_spectra / k_dndx instantiations (kernels.h) of one group of delta-f modes; the
// Makefile compiles this file once per group with -DIS3D_TU=<12|3|4|5>.  Grad shares its unit with
// RTA-CE: compiled in a module of its own, Grad's k_spectra came out with 35 spilled VGPRs and ran
// 11% slower (in any module that also holds another mode's kernels it allocates 155 VGPRs, no spills).
#define IS3D_KERNEL_DEFS
#include "kernels.h"

#ifndef IS3D_TU
#error "compile with -DIS3D_TU=<12|3|4|5>"
#endif

namespace is3d {
namespace kern {
#if IS3D_TU == 12
template void launch_spectra<GRAD>(dim3, size_t, hipStream_t, const SpecArgs&, int, int);
template void launch_spectra<CE>(dim3, size_t, hipStream_t, const SpecArgs&, int, int);
template void launch_dndx<GRAD>(dim3, size_t, hipStream_t, const DndxArgs&, int, int);
template void launch_dndx<CE>(dim3, size_t, hipStream_t, const DndxArgs&, int, int);
template void launch_phitab<GRAD>(hipStream_t, const PhiTabArgs&);
template void launch_phitab<CE>(hipStream_t, const PhiTabArgs&);
#elif IS3D_TU == 3 || IS3D_TU == 4
template void launch_spectra<IS3D_TU>(dim3, size_t, hipStream_t, const SpecArgs&, int, int);
template void launch_dndx<IS3D_TU>(dim3, size_t, hipStream_t, const DndxArgs&, int, int);
#elif IS3D_TU == 5      // operation 0 has no PTMA path (SpacetimeDistribution.cpp)
template void launch_spectra<PTMA>(dim3, size_t, hipStream_t, const SpecArgs&, int, int);
#else
#error "unknown IS3D_TU"
#endif
}  // namespace kern
}  // namespace is3d

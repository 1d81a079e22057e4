// engine.hip -- MI355X (gfx950) Cooper-Frye continuous-spectra engine behind the
// C ABI of include/is3d_amd.h.
//
// Hot path (reference MomentumSpectra.cpp:32-1682, dispatched from
// EmissionFunction.cpp:1198-1226):
//   k_prep_*      one thread per freeze-out cell: u^tau, pi^{mu nu} reconstruction,
//                 delta-f coefficients (GSL-equivalent spline / bilinear table on
//                 device), LRF basis, A^{-1} (PTM/PTB), breakdown tests -> cell record
//   k_aniso       PTMA only: one wavefront per warm-start chain (or per cell),
//                 Newton solve for (lambda, aT, aL) + famod coefficients
//   k_renorm      PTM only: per (cell, species) renormalisation n_linear / n_mod
//   k_spectra     the (cell x species x pT x phi x y [x eta]) integral: workgroup =
//                 one pT value x 256 (species, y) lanes x a cell range; each lane keeps
//                 32 phi accumulators in VGPRs; per cell tile the per-(cell,phi) and
//                 per-(cell,y/eta) factors are built cooperatively in LDS (see
//                 cf_math.h for the factorisation); no atomics, fixed summation order
//   k_reduce      sum of the cell-split partial slabs x (2 pi hbarc)^-3 x g
#ifndef IS3D_LDS_QROW_LIMIT
#define IS3D_LDS_QROW_LIMIT (80 * 1024)   // above this k_spectra takes the F_LY launch (per-lane y-term rows)
#endif
#ifndef IS3D_ANISO_MERGE
#define IS3D_ANISO_MERGE 1    // PTMA Newton sums over hadrons merged by identical (mass, sign)
#endif
#ifndef IS3D_MP
#define IS3D_MP 1             // k_spectra's F_MP launch (several pT per workgroup) for few lane tasks per pT
#endif
#ifndef IS3D_FILL_WGS
#define IS3D_FILL_WGS 8192    // k_spectra workgroups the cell splits aim for (>= 8k fills the chip evenly)
#endif
#ifndef IS3D_FILL_WGS_MP
#define IS3D_FILL_WGS_MP 2048 // the same for F_MP launches
#endif
#ifndef IS3D_CHAIN_L
#define IS3D_CHAIN_L 32       // PTMA warm-start chains: positions per segment (k_chain_pass), at least
#endif
#ifndef IS3D_CHAIN_SLOTS
#define IS3D_CHAIN_SLOTS 16384   // PTMA chain segments per pass (one wavefront each)
#endif
#ifndef IS3D_CHAIN_W
#define IS3D_CHAIN_W 4        // PTMA chain segments: wavefronts per segment sharing each Newton evaluation's terms
#endif
#ifndef IS3D_NEWTON_WAVES
#define IS3D_NEWTON_WAVES 0   // PTMA Newton kernels (k_aniso, k_chain_pass): waves per SIMD to allocate for (0: compiler)
#endif
#ifndef IS3D_MAX_SPLITS
#define IS3D_MAX_SPLITS 1024  // cap on k_spectra's cell splits (one output-sized slab each)
#endif
#ifndef IS3D_SLAB_BYTES
#define IS3D_SLAB_BYTES (48L << 30)   // ... and on their slabs' memory: config 4 (10^6 cells, 50 MB slabs) runs 880 splits
                                      // of 0.5 MB of records (44 GB of slabs): 2569 ms per pass, 512 splits 2679 ms,
                                      // 256 splits 2751 ms (profiles/round4_r4a_ab_ts.log)
#endif
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <map>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/is3d_amd.h"
#include "aniso_math.h"
#include "cf_math.h"
#include "spline_host.h"
#include "kernels.h"
#include "group.h"

using namespace is3d;
using namespace is3d::kern;

namespace {

struct DevTables {            // device copy of the delta-f tables (pointers into one blob)
  DfTables tb;
};

// ------------------------------------------------------------------------------------------
// prepass kernels
// ------------------------------------------------------------------------------------------
struct PrepArgs {
  PrepConsts k;
  DfTables tb;
  const double* surf;   // [NSURF][n]
  double* rec;          // [n][NREC]
  double* aux;          // PTM/PTB: [9][n]; PTMA: [9][n] Newton inputs
  long n;               // cells held (the field stride of surf / aux)
  long c0, c1;          // cells [c0, c1) prepared by this launch
  int* err;
  unsigned long long* cnt;  // [0] breakdown [1] pl<0 [2] recon fail [3] iterations
};

template <int MODE>
__global__ __launch_bounds__(256) void k_prep(PrepArgs A) {
  const long c = A.c0 + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= A.c1) return;
  double s[NSURF];
#pragma unroll
  for (int f = 0; f < NSURF; f++) s[f] = A.surf[(long)f * A.n + c];
  double R[NREC];
  int err = DF_OK;
  if (MODE == GRAD || MODE == CE) {
    err = prep_grad_ce(A.k, A.tb, s, R);
  } else if (MODE == PTM || MODE == PTB) {
    double aux[9];
    int flags[2];
    err = prep_feqmod(A.k, A.tb, s, R, aux, flags);
    if (!err) {
#pragma unroll
      for (int f = 0; f < 9; f++) A.aux[(long)f * A.n + c] = aux[f];
      if (flags[0] && R[R_KIND] != 0.0) atomicAdd(&A.cnt[0], 1ull);
      if (flags[1]) atomicAdd(&A.cnt[1], 1ull);
    }
  } else {
    double ain[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    prep_famod_a(A.k, s, R, ain);
#pragma unroll
    for (int f = 0; f < 9; f++) A.aux[(long)f * A.n + c] = ain[f];
  }
  if (err) { atomicMax(A.err, err); R[R_KIND] = 0.0; }
  if (R[R_KIND] != 0.0) sep_cell_consts(MODE, R);
  // Grad / RTA-CE: cells whose lanes may leave the fast path (|mu_B| / T beyond ~300) counted in cnt[4]: any such
  // cell sends the launch to the F_TB kernels, the F_TS ones carry no slow loop (launch_end)
  if (MODE <= CE && A.k.operation == 1 && R[R_KIND] != 0.0 && sep_slow_cell(R, A.k.pT_max, A.k.b_max))
    atomicAdd(&A.cnt[4], 1ULL);
#pragma unroll
  for (int f = 0; f < NREC; f++) A.rec[c * NREC + f] = R[f];
}

struct WaveSum {
  __device__ double operator()(double v) const {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  }
};

// sum over the W wavefronts of a workgroup (W x 64 lanes share one cell's Newton terms): each wave's sums, then the
// W partials from LDS in wave order (every lane gets the same bits), two barriers per red_all call of up to kRedN
// values
constexpr int kRedN = 8;
template <int W>
struct BlockSum {
  double* s;   // LDS, kRedN x W doubles
  __device__ double operator()(double v) const;
};
template <int W, class... T>
__device__ __forceinline__ void red_all(const BlockSum<W>& r, T&... v) {
  static_assert(sizeof...(T) <= kRedN, "BlockSum: at most kRedN values per call");
  ((v = WaveSum()(v)), ...);
  if constexpr (W > 1) {
    const int wave = threadIdx.x >> 6;
    int k = 0;
    if ((threadIdx.x & 63) == 0) ((r.s[(k++) * W + wave] = v), ...);
    __syncthreads();
    k = 0;
    auto sum = [&](int kk) {
      double a = r.s[kk * W];
#pragma unroll
      for (int w = 1; w < W; w++) a += r.s[kk * W + w];
      return a;
    };
    ((v = sum(k++)), ...);
    __syncthreads();
  }
}
template <int W>
__device__ double BlockSum<W>::operator()(double v) const {
  red_all(*this, v);
  return v;
}

struct AnisoArgs {
  const double* rec; const double* ain; double* sol;   // rec [n][NREC], ain [9][stride], sol [6][stride]
  long c0, n, chains;   // cells [c0, c0 + n) in `chains` warm-start chains
  long stride;          // cells held
  Hadrons h;
  double fp2;
  unsigned long long* cnt;
};

// one wavefront per warm-start chain: cells chain, chain + C, chain + 2C, ... (MomentumSpectra.cpp:98-107)
__global__ __launch_bounds__(64, IS3D_NEWTON_WAVES ? IS3D_NEWTON_WAVES : 1) void k_aniso(AnisoArgs A) {
  const long chain = blockIdx.x;
  const int lane = threadIdx.x;
  __shared__ double s_etab[kExpTabN];                       // aniso_math.h aexp (IS3D_ANISO_FAST)
  for (int i = lane; i < kExpTabN; i += 64) s_etab[i] = kExp2Tab[i];
  __syncthreads();
  Hadrons h = A.h;
  h.etab = s_etab;
  double state[4] = {0.0, 0.0, 0.0, 0.0};
  long cnt[3] = {0, 0, 0};
  for (long c = A.c0 + chain; c < A.c0 + A.n; c += A.chains) {
    if (A.rec[c * NREC + R_KIND] == 0.0) continue;
    double ain[4];
#pragma unroll
    for (int f = 0; f < 4; f++) ain[f] = A.ain[(long)f * A.stride + c];
    double out[6];
    aniso_cell(ain, h, lane, 64, WaveSum(), A.fp2, state, out, cnt);
    if (lane == 0) {
#pragma unroll
      for (int f = 0; f < 6; f++) A.sol[(long)f * A.stride + c] = out[f];
    }
  }
  if (lane == 0) {
    if (cnt[0]) atomicAdd(&A.cnt[1], (unsigned long long)cnt[0]);
    if (cnt[1]) atomicAdd(&A.cnt[2], (unsigned long long)cnt[1]);
    if (cnt[2]) atomicAdd(&A.cnt[3], (unsigned long long)cnt[2]);
  }
}

// ---- PTMA warm-start chains (MomentumSpectra.cpp:1308-1364) in parallel segments -----------------------
// The reference warm-starts each cell's Newton solve from the chain state the previous cell of its OpenMP
// thread left (chain c = cells c, c + C, c + 2C, ...; the shipped serial build is one chain).  That state
// recurrence is serial, and a lone wavefront walking it is latency-bound (354 us per cell on MI355X:
// 1e5 cells took 35 s).  The chain is instead cut into segments of L positions, one wavefront each:
//   pass 0      every segment runs its cells from a cold start (exact for each chain's first segment);
//   pass j >= 1 a segment whose incoming state (the end state the previous segment left in pass j - 1)
//               differs bitwise from the start its stored run used re-runs from the new start, and stops
//               at the first cell whose new chain state equals the stored one: from there on the stored
//               cells were computed from that same state, so they stand.  A segment that reaches its end
//               without re-synchronising publishes a new end state and flags pass j as changed.
// The passes stop once a pass changes nothing; then every segment's stored run starts from its
// predecessor's true end state, i.e. the stored states and solutions are the serial chain's, bit for bit.
// A chain state differs from a cold-start guess for ~10 cells on average before the Newton solves forget it
// (CPU sweep study, tests/native/cf_emulator.cpp emu_chain_sweeps), so a pass re-runs little.  After
// kChainPasses passes a single-wavefront finisher completes any remaining ripple serially (exact).
constexpr int kChainPasses = 24;

struct ChainArgs {
  const double* rec; const double* ain; double* sol;   // ain [9][n], sol [6][n]
  double* sta;           // [4][n] chain state after each cell (prev_ok, lambda, aT, aL)
  int* info;             // [n] Newton iterations | pl/pt < 0 << 16 | reconstruction failure << 17
  double* send;          // [2][4][nseg] segment end states, by pass parity
  double* sstart;        // [4][nseg] the start state of each segment's stored run
  int* changed;          // [kChainPasses] pass j changed some segment's end state
  long n, C, L, nspc;    // cells, chains, positions per segment, segments per chain
  // positions [q0, q1) of every chain (cells [q0 C, q1 C)): the whole chain on one engine; a device group's shard
  // solves its own range, starting each chain from the end state its predecessor shard pushes into bin
  long q0, q1;
  int has_pred;          // q0 > 0: chain position q0 - 1 lives on the previous shard
  int npass;             // passes enqueued (<= kChainPasses)
  double* bin;           // [3][4 C + 1] boundary in: end states of position q0 - 1 by pass parity, [2] = final + walk flag
  double* bout;          // [3][4 C + 1] boundary out: this range's end states (position q1 - 1), same slots
  Hadrons h;
  double fp2;
};
constexpr int kBndSlots = 3;   // bin / bout slots: pass parity 0, 1 and the finisher's

__device__ __forceinline__ bool state_eq(const double* a, const double* b) {
  bool eq = true;
#pragma unroll
  for (int f = 0; f < 4; f++) eq = eq && (__double_as_longlong(a[f]) == __double_as_longlong(b[f]));
  return eq;
}

// Run segment `seg` from `state` (its start): re-run mode (sync) stops at the first cell whose new state equals
// the stored one and returns true (end state unchanged); otherwise the state after the last cell is in `state`.
__device__ bool chain_segment_run(const ChainArgs& A, Hadrons h, long seg, double* state, bool sync) {
  const int lane = threadIdx.x;
  __shared__ double s_red[kRedN * IS3D_CHAIN_W];
  const long c = seg / A.nspc, s = seg % A.nspc;
  const long P = min((A.n - c + A.C - 1) / A.C, A.q1);      // positions of chain c in this range's end
  const long p0 = A.q0 + s * A.L, p1 = min(P, p0 + A.L);
  for (long pos = p0; pos < p1; pos++) {
    const long cell = c + pos * A.C;
    if (A.rec[cell * NREC + R_KIND] == 0.0) continue;       // u.dsigma <= 0: not in the chain (:1146)
    double ain[4];
#pragma unroll
    for (int f = 0; f < 4; f++) ain[f] = A.ain[(long)f * A.n + cell];
    // the stored state is read before the solve: its barriers keep lane 0's store below from racing a lagging
    // wavefront's read
    double old[4];
#pragma unroll
    for (int f = 0; f < 4; f++) old[f] = A.sta[(long)f * A.n + cell];
    double out[6];
    long cnt[3] = {0, 0, 0};
    aniso_cell(ain, h, lane, 64 * IS3D_CHAIN_W, BlockSum<IS3D_CHAIN_W>{s_red}, A.fp2, state, out, cnt);
    const bool same = sync && state_eq(state, old);
    if (lane == 0) {
#pragma unroll
      for (int f = 0; f < 6; f++) A.sol[(long)f * A.n + cell] = out[f];
#pragma unroll
      for (int f = 0; f < 4; f++) A.sta[(long)f * A.n + cell] = state[f];
      A.info[cell] = (int)cnt[2] | ((int)cnt[0] << 16) | ((int)cnt[1] << 17);
    }
    if (same) return true;
  }
  return false;
}

// the chain kernels' Hadrons with the LDS exp table of aniso_math.h's aexp (filled by the whole workgroup)
__device__ __forceinline__ Hadrons chain_hadrons(const ChainArgs& A, double* s_etab) {
  for (int i = threadIdx.x; i < kExpTabN; i += blockDim.x) s_etab[i] = kExp2Tab[i];
  __syncthreads();
  Hadrons h = A.h;
  h.etab = s_etab;
  return h;
}

// one workgroup of IS3D_CHAIN_W wavefronts per segment (the lanes share each Newton evaluation's terms); every
// branch below is uniform over the workgroup (the reductions hand all lanes the same bits)
__global__ __launch_bounds__(64 * IS3D_CHAIN_W, IS3D_NEWTON_WAVES ? IS3D_NEWTON_WAVES : 1) void k_chain_pass(ChainArgs A, int pass) {
  const long seg = blockIdx.x, nseg = A.C * A.nspc;
  const long c = seg / A.nspc, s = seg % A.nspc;
  const int lane = threadIdx.x;
  const long bw = 4 * A.C + 1;
  // converged: the remaining passes are no-ops (a shard with a predecessor always checks its starts: the boundary
  // pushed in may still move)
  if (pass > 0 && A.changed[pass - 1] == 0 && !A.has_pred) return;
  __shared__ double s_etab[kExpTabN];
  const Hadrons h = chain_hadrons(A, s_etab);
  const double* prev = A.send + (long)((pass + 1) & 1) * 4 * nseg;
  double* cur = A.send + (long)(pass & 1) * 4 * nseg;
  double state[4] = {0.0, 0.0, 0.0, 0.0};                   // cold: no previous success in this chain
  bool done = false;
  if (pass > 0) {
    double st0[4], used[4];
#pragma unroll
    for (int f = 0; f < 4; f++) used[f] = A.sstart[f * nseg + seg];
    if (s == 0) {
      const double* b = A.bin + (long)((pass - 1) & 1) * bw;
#pragma unroll
      for (int f = 0; f < 4; f++) st0[f] = A.has_pred ? b[f * A.C + c] : 0.0;
    } else {
#pragma unroll
      for (int f = 0; f < 4; f++) st0[f] = prev[f * nseg + seg - 1];
    }
    if (state_eq(st0, used)) {                              // same start: the stored run stands
      done = true;
    } else {
#pragma unroll
      for (int f = 0; f < 4; f++) state[f] = st0[f];
    }
    if (IS3D_CHAIN_W > 1) __syncthreads();   // every wavefront has read sstart before lane 0 rewrites it
    if (done && lane == 0) for (int f = 0; f < 4; f++) cur[f * nseg + seg] = prev[f * nseg + seg];
  }
  if (!done) {
    if (lane == 0) for (int f = 0; f < 4; f++) A.sstart[f * nseg + seg] = state[f];
    const bool synced = chain_segment_run(A, h, seg, state, pass > 0);
    if (lane == 0) {
      if (synced) {
        for (int f = 0; f < 4; f++) cur[f * nseg + seg] = prev[f * nseg + seg];
      } else {
        bool moved = pass == 0;
        for (int f = 0; f < 4; f++) {
          moved = moved || __double_as_longlong(state[f]) != __double_as_longlong(prev[f * nseg + seg]);
          cur[f * nseg + seg] = state[f];
        }
        if (moved && pass > 0) atomicOr(&A.changed[pass], 1);
      }
    }
    // pass 0 ran cold starts: exact only for the first segment of a range without a predecessor, so it flags a
    // change whenever some segment may be wrong (a finisher after a single pass must then walk)
    if (pass == 0 && lane == 0 && (A.nspc > 1 || A.has_pred)) atomicOr(&A.changed[0], 1);
  }
  // pass 0 fills both parity slots: a range without a predecessor and with one segment per chain is exact after
  // pass 0 and flags nothing, so passes 1.. return early above and never write slot 1 -- which the finisher's
  // no-walk copy and the successor shard's odd-pass boundary read
  if (pass == 0 && lane == 0) {
    double* other = A.send + 4 * nseg;
    for (int f = 0; f < 4; f++) other[f * nseg + seg] = cur[f * nseg + seg];
  }
  // the range's last segment of chain c: its end state is the next shard's boundary in
  if (s == A.nspc - 1 && lane == 0) {
    for (int slot = pass & 1; slot <= (pass == 0 ? 1 : (pass & 1)); slot++) {
      double* b = A.bout + (long)slot * bw;
      for (int f = 0; f < 4; f++) b[f * A.C + c] = cur[f * nseg + seg];
    }
  }
}

// Serial completion after the passes (one wavefront; normally returns at once): segments in chain order, each
// from its predecessor's current end state -- exact by induction.  It walks when this range's last pass changed
// something or the predecessor shard walked (bin[2] flag); either way it leaves the range's final end states and
// its walk flag in bout[2] for the next shard.
__global__ __launch_bounds__(64 * IS3D_CHAIN_W) void k_chain_finish(ChainArgs A) {
  const long nseg = A.C * A.nspc, bw = 4 * A.C + 1;
  double* cur = A.send + (long)((A.npass - 1) & 1) * 4 * nseg;
  const double* bfin = A.bin + 2 * bw;
  double* bo = A.bout + 2 * bw;
  const int lane = threadIdx.x;
  const bool walk = A.changed[A.npass - 1] != 0 || (A.has_pred && bfin[4 * A.C] != 0.0);
  if (!walk) {
    if (lane == 0) {
      for (long c = 0; c < A.C; c++)
        for (int f = 0; f < 4; f++) bo[f * A.C + c] = cur[f * nseg + c * A.nspc + A.nspc - 1];
      bo[4 * A.C] = 0.0;
    }
    return;
  }
  __shared__ double s_etab[kExpTabN];
  const Hadrons h = chain_hadrons(A, s_etab);
  // the running end state stays in registers (uniform over the wavefront): no memory round trip between
  // segments, and every array element this kernel reads was written by an earlier launch or not at all
  double carry[4] = {0.0, 0.0, 0.0, 0.0};
  for (long seg = 0; seg < nseg; seg++) {
    const long c = seg / A.nspc, s = seg % A.nspc;
    if (s == 0) {
#pragma unroll
      for (int f = 0; f < 4; f++) carry[f] = A.has_pred ? bfin[f * A.C + c] : 0.0;
    }
    double used[4];
#pragma unroll
    for (int f = 0; f < 4; f++) used[f] = A.sstart[f * nseg + seg];
    const bool same = state_eq(carry, used);
    if (IS3D_CHAIN_W > 1) __syncthreads();   // every wavefront has read sstart before lane 0 rewrites it
    if (same) {
#pragma unroll
      for (int f = 0; f < 4; f++) carry[f] = cur[f * nseg + seg];
    } else {
      if (lane == 0) for (int f = 0; f < 4; f++) A.sstart[f * nseg + seg] = carry[f];
      double state[4] = {carry[0], carry[1], carry[2], carry[3]};
      if (chain_segment_run(A, h, seg, state, true)) {
#pragma unroll
        for (int f = 0; f < 4; f++) carry[f] = cur[f * nseg + seg];
      } else {
#pragma unroll
        for (int f = 0; f < 4; f++) carry[f] = state[f];
        if (lane == 0) for (int f = 0; f < 4; f++) cur[f * nseg + seg] = state[f];
      }
    }
    if (s == A.nspc - 1 && lane == 0) for (int f = 0; f < 4; f++) bo[f * A.C + c] = carry[f];
  }
  if (lane == 0) bo[4 * A.C] = 1.0;
}

// the serial chain's counters from the per-cell records: [1] pl/pt < 0, [2] reconstruction failures,
// [3] Newton iterations
__global__ __launch_bounds__(256) void k_chain_count(const double* rec, const int* info, long c_lo, long c_hi,
                                                     unsigned long long* cnt) {
  __shared__ unsigned long long s[3][256];
  unsigned long long a = 0, b = 0, it = 0;
  for (long c = c_lo + (long)blockIdx.x * 256 + threadIdx.x; c < c_hi; c += (long)gridDim.x * 256) {
    if (rec[c * NREC + R_KIND] == 0.0) continue;
    const int v = info[c];
    it += (unsigned)(v & 0xffff); a += (v >> 16) & 1; b += (v >> 17) & 1;
  }
  s[0][threadIdx.x] = a; s[1][threadIdx.x] = b; s[2][threadIdx.x] = it;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o)
      for (int k = 0; k < 3; k++) s[k][threadIdx.x] += s[k][threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (s[0][0]) atomicAdd(&cnt[1], s[0][0]);
    if (s[1][0]) atomicAdd(&cnt[2], s[1][0]);
    if (s[2][0]) atomicAdd(&cnt[3], s[2][0]);
  }
}

__global__ __launch_bounds__(256) void k_famod_b(PrepArgs A, const double* sol) {
  const long c = A.c0 + (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= A.c1) return;
  if (A.rec[c * NREC + R_KIND] == 0.0) return;
  double R[NREC], ain[9], so[6];
#pragma unroll
  for (int f = 0; f < NREC; f++) R[f] = A.rec[c * NREC + f];
#pragma unroll
  for (int f = 0; f < 9; f++) ain[f] = A.aux[(long)f * A.n + c];
#pragma unroll
  for (int f = 0; f < 6; f++) so[f] = sol[(long)f * A.n + c];
  int broken = 0;
  prep_famod_b(A.k, R, ain, so, &broken);
  if (broken) atomicAdd(&A.cnt[0], 1ull);
#pragma unroll
  for (int f = 0; f < NREC; f++) A.rec[c * NREC + f] = R[f];
}

struct RenormArgs {
  PrepConsts k;
  const double* rec; const double* aux; double* renorm;   // renorm[c - c0][class]
  const double *mass, *sign, *degen, *baryon;              // sorted species
  const int* rrep;                                         // representative sorted species of each class
  long c0, n, stride; int npart;                           // cells [c0, c0 + n) of stride held; npart = classes
};

__global__ __launch_bounds__(256) void k_renorm(RenormArgs A) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= A.n * A.npart) return;
  const long c = A.c0 + idx / A.npart;
  const int s = A.rrep[(int)(idx % A.npart)];
  if (A.rec[c * NREC + R_KIND] == 0.0) { A.renorm[idx] = 0.0; return; }
  double aux[9];
#pragma unroll
  for (int f = 0; f < 9; f++) aux[f] = A.aux[(long)f * A.stride + c];
  A.renorm[idx] = ptm_renorm(A.k, aux, A.mass[s], A.sign[s], A.degen[s], A.baryon[s]);
}

// per-cell cost estimate (is3d_cell_costs) from the prepared records
__global__ __launch_bounds__(256) void k_cell_cost(const double* rec, long n, double fb_cost, double* cost) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const double* R = rec + c * NREC;
  const bool fb = R[R_KIND] == 1.0 || (R[R_KIND] == 2.0 && R[R_NARROW] != 0.0);
  cost[c] = R[R_KIND] == 0.0 ? kSkipCost : (fb_cost > 0.0 && fb) ? fb_cost : 1.0;
}

// Modified modes: the cells whose lanes may take the separable fallback (breakdown: R_KIND == 1; narrow
// rapidity windows: R_NARROW != 0, MomentumSpectra.cpp:863-871), listed in ascending order for the F_FB
// launch.  kFbBlocks workgroups each own a contiguous cell range: k_fbcount counts each range's cells, k_fbwrite
// writes them in order after the counts of the ranges before it (wave ballots + an LDS prefix per 256 cells) --
// deterministic, and no host round trip (the count stays on the device).  (One workgroup walking per-thread chunks
// took 44 ms per config-5 pass, 5e6 cells.)
constexpr int kFbBlocks = 1024;

__device__ __forceinline__ bool fb_cell(const double* rec, long c) {
  const double* R = rec + c * NREC;
  return R[R_KIND] == 1.0 || (R[R_KIND] == 2.0 && R[R_NARROW] != 0.0);
}

__global__ __launch_bounds__(256) void k_fbcount(const double* rec, long n, int* bcnt) {
  const long ch = (n + kFbBlocks - 1) / kFbBlocks, lo = min(n, (long)blockIdx.x * ch), hi = min(n, lo + ch);
  int cnt = 0;
  for (long c = lo + threadIdx.x; c < hi; c += 256) cnt += fb_cell(rec, c) ? 1 : 0;
  __shared__ int s[256];
  s[threadIdx.x] = cnt;
  __syncthreads();
  for (int d = 128; d > 0; d >>= 1) {
    if (threadIdx.x < d) s[threadIdx.x] += s[threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x == 0) bcnt[blockIdx.x] = s[0];
}

__global__ __launch_bounds__(256) void k_fbwrite(const double* rec, long n, const int* bcnt, int* cells, int* count) {
  const long ch = (n + kFbBlocks - 1) / kFbBlocks, lo = min(n, (long)blockIdx.x * ch), hi = min(n, lo + ch);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  __shared__ int s_base, s_w[4];
  if (t == 0) {
    int o = 0;
    for (int b = 0; b < (int)blockIdx.x; b++) o += bcnt[b];
    s_base = o;
    if (blockIdx.x == kFbBlocks - 1) *count = o + bcnt[blockIdx.x];
  }
  __syncthreads();
  for (long c0 = lo; c0 < hi; c0 += 256) {
    const long c = c0 + t;
    const bool f = c < hi && fb_cell(rec, c);
    const unsigned long long m = __ballot(f);
    if (lane == 0) s_w[wave] = __popcll(m);
    __syncthreads();
    int o = s_base;
    for (int w = 0; w < wave; w++) o += s_w[w];
    if (f) cells[o + __popcll(m & ((1ull << lane) - 1ull))] = (int)c;
    __syncthreads();
    if (t == 0) s_base += s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
  }
}

// the ascending fallback-cell list of nw records into list[1 ..], its length into list[0]; list holds nw + 1 +
// kFbBlocks ints (the per-range counts after the list)
static void enqueue_fbscan(const double* rec, long nw, int* list, hipStream_t st) {
  int* bcnt = list + 1 + nw;
  hipLaunchKernelGGL(k_fbcount, dim3(kFbBlocks), dim3(256), 0, st, rec, nw, bcnt);
  hipLaunchKernelGGL(k_fbwrite, dim3(kFbBlocks), dim3(256), 0, st, rec, nw, (const int*)bcnt, list + 1, list);
}

struct ReduceArgs {
  const double* slab; long sstride; int nsplit;
  int nbx, npart, npT, nphi, nk, nl, ny_out, kj; long ntask;   // npart: lane species (integrand classes)
  const int* sorig; const double* degen_orig; double prefactor;
  const int *cmem_off, *cmem;   // member sorted species of each class
  double* out;
  const unsigned long long* gate; int gate_want;   // launch_end's device-side plan choice (kernels.h SpecArgs)
};

// every member species of class c gets (2 pi hbarc)^-3 g_s x the class's sum
__device__ __forceinline__ void write_members(const ReduceArgs& A, int c, long off, double acc, int m0, int dm) {
  for (int m = A.cmem_off[c] + m0; m < A.cmem_off[c + 1]; m += dm) {
    const int so = A.sorig[A.cmem[m]];
    A.out[(long)so * A.npT * A.nphi * A.ny_out + off] = A.prefactor * A.degen_orig[so] * acc;
  }
}

// dN[s][pT][phi][y] = (2 pi hbarc)^-3 g_s * sum over eta nodes (2+1D) and cell splits, in fixed order.
// One thread per slab entry of an l = 0 lane; the lanes of the other eta nodes of the same (class, y,
// phi block) are task + l * npart.
__global__ __launch_bounds__(256) void k_reduce(ReduceArgs A) {
  if (gate_closed(A.gate, A.gate_want)) return;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= A.sstride) return;
  const int KJ = A.kj;
  const int lane = (int)(e % kBlock);
  const int jj = (int)((e / kBlock) % KJ);
  const long rest = e / ((long)kBlock * KJ);
  const int lane_group = (int)(rest % A.nbx), ipt = (int)(rest / A.nbx);
  const long task = (long)lane_group * kBlock + lane;
  if (task >= A.ntask) return;
  const int s = (int)(task % A.npart);
  const long r = task / A.npart;
  const long nq = (long)A.nk * A.nl;
  const int q = (int)(r % nq);
  if (q % A.nl != 0) return;
  const int k = q / A.nl, j = (int)(r / nq) * KJ + jj;
  if (j >= A.nphi) return;
  double acc = 0.0;
  for (int l = 0; l < A.nl; l++) {
    const long tl = task + (long)l * A.npart;
    const long el = ((long)ipt * A.nbx + tl / kBlock) * ((long)KJ * kBlock) + (long)jj * kBlock + tl % kBlock;
    for (int z = 0; z < A.nsplit; z++) acc += A.slab[(long)z * A.sstride + el];
  }
  write_members(A, s, ((long)ipt * A.nphi + j) * A.ny_out + k, acc, 0, 1);
}

// The same sum with one wavefront per output entry, for slabs with many (eta node, cell split) terms per
// output (2+1D: 24 eta nodes x hundreds of splits -- the per-thread loop above ran 8k dependent loads per
// output and took 2.4 ms for pikp 1e5 cells): lane i adds terms i, i + 64, ... of the (l, split) list,
// then a fixed xor-shuffle tree combines the lanes, so the order stays fixed (bit-reproducible).
__global__ __launch_bounds__(256) void k_reduce_wave(ReduceArgs A) {
  if (gate_closed(A.gate, A.gate_want)) return;
  const long o = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long nout = (long)A.npart * A.npT * A.nphi * A.ny_out;
  if (o >= nout) return;                                   // whole wavefronts exit together
  const int k = (int)(o % A.ny_out);
  const long r1 = o / A.ny_out;
  const int j = (int)(r1 % A.nphi);
  const long r2 = r1 / A.nphi;
  const int ipt = (int)(r2 % A.npT), s = (int)(r2 / A.npT);
  const int KJ = A.kj, jb = j / KJ, jj = j % KJ;
  const long nq = (long)A.nk * A.nl;
  const long task0 = s + (long)A.npart * (k * A.nl + nq * jb);
  const long nterm = (long)A.nl * A.nsplit;
  double acc = 0.0;
  for (long m = lane; m < nterm; m += 64) {
    const int l = (int)(m / A.nsplit), z = (int)(m % A.nsplit);
    const long tl = task0 + (long)l * A.npart;
    const long el = ((long)ipt * A.nbx + tl / kBlock) * ((long)KJ * kBlock) + (long)jj * kBlock + tl % kBlock;
    acc += A.slab[(long)z * A.sstride + el];
  }
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) acc += __shfl_xor(acc, w, 64);
  write_members(A, s, ((long)ipt * A.nphi + j) * A.ny_out + k, acc, lane, 64);
}

// Chunk-wise slab fold (folded F_TS launches, enqueue_spectra): acc[i] = (init ? 0 : acc[i]) + src[0][i] + ... +
// src[ns - 1][i], added in split order, so the folded accumulator equals k_reduce's sequential sum over all splits
// bit for bit (3+1D: one term per split and output).  Memory-bound: ns + 2 doubles per entry.
__global__ __launch_bounds__(256) void k_fold(double* acc, const double* src, long sstride, int ns, int init,
                                              const unsigned long long* gate, int gate_want) {
  if (gate_closed(gate, gate_want)) return;      // the other plan of a gated pair runs (launch_end)
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < sstride; i += (long)gridDim.x * blockDim.x) {
    double a = init ? 0.0 : acc[i];
    for (int z = 0; z < ns; z++) a += src[(long)z * sstride + i];
    acc[i] = a;
  }
}

// per-cell spacetime bin indices (SpacetimeDistribution.cpp:380-392): keys[0..2][c] = itau, ir, iphi (-1 outside)
struct KeyArgs {
  const double *tau, *x, *y; long n;
  double tau_min, tau_width, r_min, r_width, phip_width;
  int tau_bins, r_bins, phip_bins;
  int* keys;
};

__global__ __launch_bounds__(256) void k_stkeys(KeyArgs A) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= A.n) return;
  const double two_pi = 2.0 * M_PI;
  const double x = A.x[c], y = A.y[c], tau = A.tau[c];
  const double r = sqrt(x * x + y * y);
  double phi = atan2(y, x);
  if (phi < 0.0) phi += two_pi;
  const long itau = (int)floor((tau - A.tau_min) / A.tau_width);
  const long ir = (int)floor((r - A.r_min) / A.r_width);
  const long iphi = (int)floor(phi / A.phip_width);
  A.keys[c] = (itau >= 0 && itau < A.tau_bins) ? (int)itau : -1;
  A.keys[A.n + c] = (ir >= 0 && ir < A.r_bins) ? (int)ir : -1;
  A.keys[2 * A.n + c] = (iphi >= 0 && iphi < A.phip_bins) ? (int)iphi : -1;
}

// part[s_orig][e] = prefactor g_s x sum over the cells of entry e = (distribution, thread slice n, bin),
// cells in ascending order (the reference's per-thread order); perm/offs: CSR built on the host
struct BinArgs {
  const double* ycell; long n; int npart;          // ycell: [class][n]; npart sorted species
  const int *perm; const long* offs; long nent;
  const int* sorig; const double* sdegen; double prefactor;
  const int* scls;                                  // sorted species -> integrand class
  double* part;
};

__global__ __launch_bounds__(256) void k_stbin(BinArgs A) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= A.nent * A.npart) return;
  const int s = (int)(idx / A.nent);
  const long e = idx % A.nent;
  const double f = A.prefactor * A.sdegen[s];
  double acc = 0.0;
  for (long i = A.offs[e]; i < A.offs[e + 1]; i++) {
    acc += f * A.ycell[(long)A.scls[s] * A.n + A.perm[i]];
  }
  A.part[(long)A.sorig[s] * A.nent + e] = acc;
}

// ------------------------------------------------------------------------------------------
// operation = 2 oversampling estimate (ParticleSampler.cpp:447-636, DeltafData.cpp:555-690)
// ------------------------------------------------------------------------------------------
struct DensArgs {
  DfTables tb;
  const double *gla;              // [alpha][pts] roots then [alpha][pts] weights
  int gla_alpha, gla_pts;
  double T, E, P, muB, nB;        // Plasma averages
  const double *smass, *ssign, *sdegen, *sbaryon; const int* sorig;
  int npart, df_mode;
  double two_pi2_hbarC3;
  double* dens;                   // [3][npart] original species order
  int* err;
};

// one wavefront per (mass-sorted) species: lane k holds Gauss-Laguerre node k of each alpha
__global__ __launch_bounds__(64) void k_densities(DensArgs A) {
  const int s = blockIdx.x, lane = threadIdx.x;
  DfCoef df;
  const int err = df_eval(A.tb, A.T, A.muB, A.E, A.P, 0.0, df);     // DeltafData.cpp:574
  if (err) { if (lane == 0) atomicMax(A.err, err); return; }
  const double mass = A.smass[s], sign = A.ssign[s], baryon = A.sbaryon[s];
  const double mbar = mass / A.T, chem = baryon * (A.muB / A.T);
  const double* W = A.gla + (long)A.gla_alpha * A.gla_pts;
  static constexpr int kAlpha[6] = {1, 1, 1, 2, 3, 3};
  double J[6];
  WaveSum ws;
#pragma unroll
  for (int q = 0; q < 6; q++) {
    double v = 0.0;
    for (int k = lane; k < A.gla_pts; k += 64) {
      const long o = (long)kAlpha[q] * A.gla_pts + k;
      v += W[o] * gt_term(q, A.gla[o], mbar, chem, sign);
    }
    J[q] = ws(v);
  }
  if (lane == 0) {
    double d3[3];
    species_densities(A.df_mode, df, A.T, A.nB / (A.E + A.P), mass, A.sdegen[s], baryon, J, A.two_pi2_hbarC3, d3);
    const int so = A.sorig[s];
    for (int i = 0; i < 3; i++) A.dens[(long)i * A.npart + so] = d3[i];
  }
}

struct YieldArgs {
  PrepConsts k;
  DfTables tb;
  const double* surf; long n;
  const double* dens; int npart;
  double* partial;                // [gridDim.x] per-block sums
  int* err;
};

// one thread per cell, fixed-order tree sum per block (bit-reproducible); the host adds the blocks in order
__global__ __launch_bounds__(256) void k_yield(YieldArgs A) {
  __shared__ double red[256];
  __shared__ double dsum[3];
  const int tid = threadIdx.x;
  if (tid < 3) {                  // species sums in species order
    double a = 0.0;
    for (int i = 0; i < A.npart; i++) a += A.dens[(long)tid * A.npart + i];
    dsum[tid] = a;
  }
  __syncthreads();
  const long c = (long)blockIdx.x * 256 + tid;
  double v = 0.0;
  if (c < A.n) {
    double sv[NSURF];
#pragma unroll
    for (int f = 0; f < NSURF; f++) sv[f] = A.surf[(long)f * A.n + c];
    const int err = yield_cell(A.k, A.tb, sv, dsum, &v);
    if (err) { atomicMax(A.err, err); v = 0.0; }
  }
  red[tid] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) red[tid] += red[tid + o];
    __syncthreads();
  }
  if (tid == 0) A.partial[blockIdx.x] = red[0];
}

// ------------------------------------------------------------------------------------------
// PTB "Jonah" table (DeltafData.cpp:220-295): thread (row, hadron) evaluates the two Gauss sums, one
// thread per row then adds the hadrons in PDG order (the reference's order), so the table is
// bit-reproducible; row kJonahN holds the lambda = 0 terms.
// ------------------------------------------------------------------------------------------
struct JonahArgs {
  double T; int npdg, pts;
  const double *mass, *degen, *sign, *r2, *w2;
  double* terms;                  // [kJonahN + 1][2][npdg]
  double *l2, *z, *bp;            // [kJonahN] each
};

__global__ __launch_bounds__(256) void k_jonah_terms(JonahArgs A) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)(kJonahN + 1) * A.npdg) return;
  const int i = (int)(idx / A.npdg), n = (int)(idx % A.npdg);
  const double lambda = (i < kJonahN) ? jonah_lambda(i) : 0.0;
  double* t = A.terms + (long)i * 2 * A.npdg;
  jonah_terms(A.T, A.mass[n], A.degen[n], A.sign[n], A.r2, A.w2, A.pts, lambda, t + n, t + A.npdg + n);
}

__global__ __launch_bounds__(64) void k_jonah_sum(JonahArgs A) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kJonahN) return;
  const double* e0 = A.terms + (long)kJonahN * 2 * A.npdg;
  const double* p0 = e0 + A.npdg;
  const double* em = A.terms + (long)i * 2 * A.npdg;
  const double* pm = em + A.npdg;
  double E = 0.0, P = 0.0, Em = 0.0, Pm = 0.0;
  for (int n = 0; n < A.npdg; n++) {
    if (A.mass[n] == 0.0) continue;
    E += e0[n]; P += p0[n]; Em += em[n]; Pm += pm[n];
  }
  jonah_row(i, E, P, Em, Pm, A.l2, A.z, A.bp);
}

__global__ void k_df_eval(DfTables tb, double T, double muB, double E, double P, double bulkPi, double* out, int* err) {
  DfCoef df;
  *err = df_eval(tb, T, muB, E, P, bulkPi, df);
  const double o[15] = {df.c0, df.c1, df.c2, df.c3, df.c4, df.shear14, df.F, df.G, df.betabulk, df.betaV, df.betapi,
                        df.lambda, df.z, df.dlambda, df.dz};
  for (int i = 0; i < 15; i++) out[i] = o[i];
}

template <class T>
T* dalloc(size_t count) {
  void* p = nullptr;
  if (count == 0) count = 1;
  if (hipMalloc(&p, count * sizeof(T)) != hipSuccess) return nullptr;
  return (T*)p;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// engine
// ------------------------------------------------------------------------------------------
// one launch's state between the stages of a staged launch (launch_begin .. launch_end)
struct LaunchCtx {
  hipStream_t st = nullptr;
  double* dev_out = nullptr;
  long wlo = 0, whi = 0, nw = 0, p0 = 0, p1 = 0;
  bool chained = false, empty = false;
  PrepArgs pa{};
  ChainArgs ca{};
};

struct is3d_engine {
  int device = 0;
  std::string err;
  // is3d_create_devices: the shard engines and their reduction (group.hip); every entry point forwards
  is3d::Group* grp = nullptr;
  // cell window [win_lo, win_hi) of the held surface that k_spectra integrates (-1: every cell); set by a
  // group whose shards hold the whole surface for the PTMA warm-start chains
  long win_lo = -1, win_hi = -1;
  // is3d_set_chain_range: PTMA warm-start chain positions [chain_q0, chain_q1) this engine solves (-1: all), for the
  // staged launch of one process per GPU
  long chain_q0 = -1, chain_q1 = -1;
  bool have_params = false, have_species = false, have_pdg = false, have_grid = false, have_gla = false, have_df = false;
  is3d_params p{};
  // species (original order) and mass-sorted permutation
  std::vector<double> mass, sign, degen, baryon;
  std::vector<int> order;
  std::vector<double> pdg_mass, pdg_sign, pdg_degen, pdg_baryon;
  std::vector<double> pT, phi, y, eta, eta_w;
  std::vector<double> pT_w, phi_w;       // operation 0 quadrature weights
  bool have_weights = false, have_bins = false;
  is3d_spacetime_bins bins{};
  int gla_alpha = 0, gla_pts = 0;
  std::vector<double> gla_r, gla_w;
  int nT = 0, nmuB = 0;
  std::vector<double> Tarr, muBarr, tab;
  double T_avg = 0.0;
  // derived host tables
  std::vector<double> jl2, jz, jx, jl2c, jzc;
  double bp_max = -1.0;
  bool tables_dirty = true;
  // device
  double* d_tables = nullptr; size_t tables_len = 0;
  DfTables dtb{};
  double* d_const = nullptr; size_t const_len = 0;    // species, grids, gla, pdg
  const double *d_smass = nullptr, *d_ssign = nullptr, *d_sbaryon = nullptr, *d_sdegen = nullptr, *d_degen_orig = nullptr;
  const double* d_csg = nullptr;   // [npT][nphp] {pT cos, pT sin}
  const double *d_pT = nullptr, *d_cphi = nullptr, *d_sphi = nullptr, *d_y = nullptr, *d_eta = nullptr, *d_etaw = nullptr;
  const double *d_pTw = nullptr, *d_phiw = nullptr;
  const double *d_gla = nullptr;
  const double *d_pdg = nullptr;
  const double* d_aniso_h = nullptr;   // [3][n_aniso_h] merged (mass, sign, degeneracy) of the PTMA hadrons
  int n_aniso_h = 0;
  int* d_sorig = nullptr;
  // PTM renormalisation classes: sorted species with identical (mass, sign, baryon) and a zero / nonzero degeneracy
  // share one n_linear / n_mod per cell (ptm_renorm depends on nothing else, ptm_gkey): d_rcls[s] = class of sorted species s,
  // d_rrep[k] = a representative sorted species of class k (SMASH 444 -> nrcls classes)
  int* d_rcls = nullptr;
  int* d_rrep = nullptr;
  int nrcls = 0;
  // integrand classes (is3d_set_species_classes, default on): the momentum integrals see a species only through
  // its (mass, sign, baryon) -- plus, in PTM, whether its degeneracy is zero (ptm_gkey) -- and the engine applies the degeneracy once, to the cell sum, in k_reduce (the reference
  // multiplies every cell's term by prefactor x degeneracy, MomentumSpectra.cpp:365: the same product up to
  // rounding), so sorted species with identical keys have bit-identical cell sums: k_spectra / k_dndx integrate one lane species per class (SMASH 444 -> 193, UrQMD 305 -> 124) and the
  // reduction writes every member.  d_cmass/d_csign/d_cbaryon: class values, d_crcls: class -> renorm class,
  // d_cmem[d_cmem_off[c] ..]: member sorted species of class c, d_scls: sorted species -> class.
  bool classes = true;
  int ncls = 0;
  std::vector<int> scls;   // host copy of d_scls
  const double *d_cmass = nullptr, *d_csign = nullptr, *d_cbaryon = nullptr;
  int *d_crcls = nullptr, *d_cmem_off = nullptr, *d_cmem = nullptr, *d_scls = nullptr;
  double* d_surf = nullptr; bool surf_owned = false; long ncell = 0; long surf_cap = 0;
  double* d_chain = nullptr; long chain_cap = 0;   // PTMA warm-start chain segments (k_chain_pass)
  double *d_rec = nullptr, *d_aux = nullptr, *d_sol = nullptr, *d_renorm = nullptr, *d_slab = nullptr, *d_out = nullptr;
  long rec_cap = 0, aux_cap = 0, sol_cap = 0, renorm_cap = 0, slab_cap = 0, out_cap = 0;
  int* d_fb = nullptr;        // modified modes: [0] fallback cell count, [1..] k_fbwrite's cell list
  long fb_cap = 0;
  double* d_phtab = nullptr;  // F_TS launches: k_phitab's per-(cell, pT, phi) rows of one chunk of cells
  long phtab_cap = 0;
  double* d_phtab2 = nullptr; // ... and of the next chunk, integrated on the side stream meanwhile
  long phtab2_cap = 0;
  hipStream_t side = nullptr; // F_TS chunks alternate between the launch stream and this one
  hipEvent_t fork = nullptr, join = nullptr;
  // folded F_TS chunks (IS3D_SLAB_FOLD): k_fold runs on its own stream, in chunk order, after each chunk's k_spectra
  // (ev_spec); a chunk reusing a slab buffer waits for the fold that emptied it (ev_fold)
  hipStream_t fold_st = nullptr;
  hipEvent_t ev_spec[2] = {nullptr, nullptr}, ev_fold[2] = {nullptr, nullptr}, fold_join = nullptr;
  // is3d_set_tuning: F_TS table chunking (defaults IS3D_PHITAB_ONE / IS3D_PHITAB_BYTES): tables of the whole window
  // up to phitab_one bytes are one chunk, larger ones chunks of whole cell splits of about phitab_chunk bytes
  long phitab_one = IS3D_PHITAB_ONE, phitab_chunk = IS3D_PHITAB_BYTES;
  long last_nchunk = 0;       // F_TS chunks of the last launch (0: not an F_TS launch)
  // is3d_set_tuning: k_spectra's cell splits (defaults IS3D_MAX_SPLITS / IS3D_SLAB_BYTES / IS3D_SPLIT_BYTES)
  long max_splits = IS3D_MAX_SPLITS, slab_bytes = IS3D_SLAB_BYTES, split_bytes = IS3D_SPLIT_BYTES;
  long last_nsplit = 0;       // cell splits of the last launch's main plan
  long last_nslab = 0;        // ... and the output-sized partial slabs it held (folded F_TS chunks: 1 + 2 spc)
  // operation 0
  double *d_ycell = nullptr, *d_part = nullptr; long ycell_cap = 0, part_cap = 0;
  int *d_keys = nullptr, *d_perm = nullptr; long keys_cap = 0, perm_cap = 0;
  long* d_offs = nullptr; long offs_cap = 0;
  long ycell_n = -1;
  int* d_err = nullptr;
  unsigned long long* d_cnt = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  LaunchCtx lc;               // the launch in flight (staged launches)
  is3d_stats st{};
  bool launched = false;

  int fail(int code, const std::string& msg) { err = msg; return code; }
};

static int hip_fail(is3d_engine* e, hipError_t h, const char* what) {
  return e->fail(IS3D_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(h));
}
#define HIPCHK(e, x)                                           \
  do {                                                         \
    hipError_t h_ = (x);                                       \
    if (h_ != hipSuccess) return hip_fail((e), h_, #x);        \
  } while (0)

static void dfree(void* p) { if (p) (void)hipFree(p); }

extern "C" int is3d_abi_version(void) { return IS3D_ABI_VERSION; }

#ifndef IS3D_BUILD_ID
#define IS3D_BUILD_ID "unknown"
#endif
extern "C" const char* is3d_build_id(void) { return IS3D_BUILD_ID; }

extern "C" is3d_engine* is3d_create(int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  is3d_engine* e = new is3d_engine();
  e->device = device;
  if (hipMalloc(&e->d_err, sizeof(int)) != hipSuccess || hipMalloc(&e->d_cnt, 8 * sizeof(unsigned long long)) != hipSuccess) {
    delete e;
    return nullptr;
  }
  for (auto& v : e->ev) (void)hipEventCreate(&v);
  return e;
}

extern "C" void is3d_destroy(is3d_engine* e) {
  if (!e) return;
  if (e->grp) {
    is3d::group_destroy(e->grp);
    delete e;
    return;
  }
  (void)hipSetDevice(e->device);
  (void)hipDeviceSynchronize();
  dfree(e->d_tables); dfree(e->d_const);
  if (e->surf_owned) dfree(e->d_surf);
  dfree(e->d_chain);
  dfree(e->d_rec); dfree(e->d_aux); dfree(e->d_sol); dfree(e->d_renorm); dfree(e->d_slab); dfree(e->d_out);
  dfree(e->d_fb); dfree(e->d_phtab); dfree(e->d_phtab2);
  if (e->side) (void)hipStreamDestroy(e->side);
  if (e->fold_st) (void)hipStreamDestroy(e->fold_st);
  for (auto v : {e->ev_spec[0], e->ev_spec[1], e->ev_fold[0], e->ev_fold[1], e->fold_join})
    if (v) (void)hipEventDestroy(v);
  if (e->fork) (void)hipEventDestroy(e->fork);
  if (e->join) (void)hipEventDestroy(e->join);
  dfree(e->d_ycell); dfree(e->d_part); dfree(e->d_keys); dfree(e->d_perm); dfree(e->d_offs);
  dfree(e->d_err); dfree(e->d_cnt);
  for (auto& v : e->ev) if (v) (void)hipEventDestroy(v);
  delete e;
}

extern "C" const char* is3d_last_error(const is3d_engine* e) {
  if (!e) return "null engine";
  return e->grp ? is3d::group_error(e->grp) : e->err.c_str();
}

extern "C" is3d_engine* is3d_create_devices(int n, const int* devices) {
  std::string err;
  is3d::Group* g = is3d::group_create(n, devices, err);
  if (!g) return nullptr;
  is3d_engine* e = new is3d_engine();
  e->device = devices[0];
  e->grp = g;
  return e;
}

extern "C" int is3d_set_cell_window(is3d_engine* e, long lo, long hi) {
  if (!e) return IS3D_ERR_ARG;
  if (e->grp) return is3d::group_fail(e->grp, IS3D_ERR_UNSUPPORTED, "a device-list engine places its own windows");
  e->chain_q0 = e->chain_q1 = -1;
  if (lo < 0 || hi < 0) { e->win_lo = e->win_hi = -1; return IS3D_OK; }
  if (lo > hi || hi > e->ncell) return e->fail(IS3D_ERR_ARG, "cell window outside the surface");
  e->win_lo = lo; e->win_hi = hi;
  return IS3D_OK;
}

extern "C" int is3d_set_tuning(is3d_engine* e, const char* key, long value) {
  if (e && e->grp) return key ? is3d::group_set_tuning(e->grp, key, value) : IS3D_ERR_ARG;
  if (!e || !key) return IS3D_ERR_ARG;
  if (!std::strcmp(key, "phitab_one_bytes")) e->phitab_one = value < 0 ? (long)IS3D_PHITAB_ONE : value;
  else if (!std::strcmp(key, "phitab_chunk_bytes")) e->phitab_chunk = value <= 0 ? (long)IS3D_PHITAB_BYTES : value;
  else if (!std::strcmp(key, "max_splits")) e->max_splits = value <= 0 ? (long)IS3D_MAX_SPLITS : value;
  else if (!std::strcmp(key, "slab_bytes")) e->slab_bytes = value <= 0 ? (long)IS3D_SLAB_BYTES : value;
  else if (!std::strcmp(key, "split_bytes")) e->split_bytes = value <= 0 ? (long)IS3D_SPLIT_BYTES : value;
  else return e->fail(IS3D_ERR_ARG, std::string("is3d_set_tuning: unknown key ") + key);
  return IS3D_OK;
}

extern "C" long is3d_get_tuning(const is3d_engine* e, const char* key) {
  if (!e || !key) return -1;
  if (e->grp) return is3d::group_get_tuning(e->grp, key);
  if (!std::strcmp(key, "phitab_one_bytes")) return e->phitab_one;
  if (!std::strcmp(key, "phitab_chunk_bytes")) return e->phitab_chunk;
  if (!std::strcmp(key, "phitab_chunks")) return e->last_nchunk;
  if (!std::strcmp(key, "max_splits")) return e->max_splits;
  if (!std::strcmp(key, "slab_bytes")) return e->slab_bytes;
  if (!std::strcmp(key, "split_bytes")) return e->split_bytes;
  if (!std::strcmp(key, "splits")) return e->last_nsplit;
  if (!std::strcmp(key, "slabs")) return e->last_nslab;
  return -1;
}

extern "C" int is3d_set_params(is3d_engine* e, const is3d_params* p) {
  if (e && e->grp) return p ? is3d::group_set_params(e->grp, p) : IS3D_ERR_ARG;
  if (!e || !p) return IS3D_ERR_ARG;
  // operation 2 is accepted for its oversampling estimate (is3d_total_yield); the sampler itself is not on this path
  if (p->operation < 0 || p->operation > 2)
    return e->fail(IS3D_ERR_ARG, "calculate_spectra error: need to set operation = (0, 1, 2)");
  if (p->dimension != 2 && p->dimension != 3) return e->fail(IS3D_ERR_ARG, "EmissionFunctionArray error: need to set dimension = (2,3)");
  if (p->df_mode < 1 || p->df_mode > 5) return e->fail(IS3D_ERR_ARG, "EmissionFunctionArray error: need to set df_mode = (1,2,3,4,5)");
  if (p->df_mode == PTB && p->include_baryon) return e->fail(IS3D_ERR_UNSUPPORTED, "Bilinear interpolation error: Jonah df doesn't work for nonzero muB. Exiting..");
  if (p->famod_chains < 0) return e->fail(IS3D_ERR_ARG, "famod_chains must be >= 0");
  e->p = *p;
  e->have_params = true;
  e->tables_dirty = true;
  return IS3D_OK;
}

extern "C" int is3d_set_species(is3d_engine* e, int n, const double* mass, const double* sign, const double* degeneracy,
                                const double* baryon) {
  if (e && e->grp) return is3d::group_set_species(e->grp, n, mass, sign, degeneracy, baryon);
  if (!e || n <= 0 || !mass || !sign || !degeneracy || !baryon) return e ? e->fail(IS3D_ERR_ARG, "bad species arrays") : IS3D_ERR_ARG;
  e->mass.assign(mass, mass + n); e->sign.assign(sign, sign + n); e->degen.assign(degeneracy, degeneracy + n);
  e->baryon.assign(baryon, baryon + n);
  e->order.resize(n);
  for (int i = 0; i < n; i++) e->order[i] = i;
  // lanes of a wavefront take consecutive species: sort by mass so that whole wavefronts hit the
  // exp-underflow early-out together (output order is unchanged)
  std::stable_sort(e->order.begin(), e->order.end(), [&](int a, int b) { return e->mass[a] < e->mass[b]; });
  e->have_species = true;
  e->tables_dirty = true;
  return IS3D_OK;
}

static int finalize_tables(is3d_engine* e);

extern "C" int is3d_set_species_classes(is3d_engine* e, int on) {
  if (e && e->grp) return is3d::group_set_species_classes(e->grp, on);
  if (!e) return IS3D_ERR_ARG;
  e->classes = on != 0;
  e->tables_dirty = true;
  return IS3D_OK;
}

extern "C" int is3d_species_integrated(is3d_engine* e) {
  if (e && e->grp) return is3d::group_species_integrated(e->grp);
  if (!e) return -IS3D_ERR_ARG;
  const int rc = finalize_tables(e);
  return rc ? -rc : e->ncls;       // an error as minus its IS3D_ERR_* code (a count is >= 1)
}

extern "C" int is3d_set_pdg(is3d_engine* e, int n, const double* mass, const double* sign, const double* degeneracy,
                            const double* baryon) {
  if (e && e->grp) return is3d::group_set_pdg(e->grp, n, mass, sign, degeneracy, baryon);
  if (!e || n <= 0 || !mass || !sign || !degeneracy || !baryon) return e ? e->fail(IS3D_ERR_ARG, "bad pdg arrays") : IS3D_ERR_ARG;
  e->pdg_mass.assign(mass, mass + n); e->pdg_sign.assign(sign, sign + n); e->pdg_degen.assign(degeneracy, degeneracy + n);
  e->pdg_baryon.assign(baryon, baryon + n);
  e->have_pdg = true;
  e->tables_dirty = true;
  return IS3D_OK;
}

extern "C" int is3d_set_momentum_grid(is3d_engine* e, int npT, const double* pT, int nphi, const double* phi, int ny,
                                      const double* y, int neta, const double* eta, const double* eta_weight) {
  if (e && e->grp) return is3d::group_set_momentum_grid(e->grp, npT, pT, nphi, phi, ny, y, neta, eta, eta_weight);
  if (!e) return IS3D_ERR_ARG;
  if (npT <= 0 || nphi <= 0 || !pT || !phi) return e->fail(IS3D_ERR_ARG, "empty pT/phi table");
  e->pT.assign(pT, pT + npT); e->phi.assign(phi, phi + nphi);
  e->y.assign(y ? y : pT, y ? y + std::max(ny, 0) : pT);
  e->eta.assign(eta ? eta : pT, eta ? eta + std::max(neta, 0) : pT);
  e->eta_w.assign(eta_weight ? eta_weight : pT, eta_weight ? eta_weight + std::max(neta, 0) : pT);
  e->have_grid = true;
  e->tables_dirty = true;
  return IS3D_OK;
}

extern "C" int is3d_set_momentum_weights(is3d_engine* e, const double* pT_weight, const double* phi_weight) {
  if (e && e->grp) return is3d::group_set_momentum_weights(e->grp, pT_weight, phi_weight);
  if (!e) return IS3D_ERR_ARG;
  if (!e->have_grid) return e->fail(IS3D_ERR_STATE, "is3d_set_momentum_grid not called");
  if (!pT_weight || !phi_weight) return e->fail(IS3D_ERR_ARG, "null pT/phi weights");
  e->pT_w.assign(pT_weight, pT_weight + e->pT.size());
  e->phi_w.assign(phi_weight, phi_weight + e->phi.size());
  e->have_weights = true;
  e->tables_dirty = true;
  return IS3D_OK;
}

extern "C" int is3d_set_spacetime_bins(is3d_engine* e, const is3d_spacetime_bins* b) {
  if (e && e->grp) return b ? is3d::group_set_spacetime_bins(e->grp, b) : IS3D_ERR_ARG;
  if (!e || !b) return IS3D_ERR_ARG;
  if (b->tau_bins <= 0 || b->r_bins <= 0 || b->phip_bins <= 0) return e->fail(IS3D_ERR_ARG, "spacetime bins must be positive");
  if (!(b->tau_max > b->tau_min) || !(b->r_max > b->r_min)) return e->fail(IS3D_ERR_ARG, "spacetime bin ranges must be increasing");
  if (b->threads < 0) return e->fail(IS3D_ERR_ARG, "spacetime threads must be >= 0");
  e->bins = *b;
  e->have_bins = true;
  return IS3D_OK;
}

extern "C" int is3d_set_gauss_laguerre(is3d_engine* e, int alpha, int points, const double* roots, const double* weights) {
  if (e && e->grp) return is3d::group_set_gauss_laguerre(e->grp, alpha, points, roots, weights);
  if (!e) return IS3D_ERR_ARG;
  if (alpha < 3 || points <= 0 || !roots || !weights) return e->fail(IS3D_ERR_ARG, "Gauss-Laguerre table needs alpha >= 3");
  e->gla_alpha = alpha; e->gla_pts = points;
  e->gla_r.assign(roots, roots + (size_t)alpha * points);
  e->gla_w.assign(weights, weights + (size_t)alpha * points);
  e->have_gla = true;
  e->tables_dirty = true;
  return IS3D_OK;
}

extern "C" int is3d_set_df_tables(is3d_engine* e, int nT, int nmuB, const double* T, const double* muB,
                                  const double* tables, double T_avg) {
  if (e && e->grp) return is3d::group_set_df_tables(e->grp, nT, nmuB, T, muB, tables, T_avg);
  if (!e) return IS3D_ERR_ARG;
  if (nT < 3 || nmuB < 1 || !T || !muB || !tables) return e->fail(IS3D_ERR_ARG, "bad df coefficient tables");
  e->nT = nT; e->nmuB = nmuB;
  e->Tarr.assign(T, T + nT); e->muBarr.assign(muB, muB + nmuB);
  e->tab.assign(tables, tables + (size_t)10 * nmuB * nT);
  e->T_avg = T_avg;
  e->have_df = true;
  e->tables_dirty = true;
  return IS3D_OK;
}

// Build the derived tables (splines, Jonah) and upload everything read-only to HBM.
// PTB Jonah table on the device (k_jonah_terms + k_jonah_sum) into e->jl2 / jz / jx / bp_max; the
// host keeps only the two 301-point spline solves
static int device_jonah_table(is3d_engine* e, const double* r2, const double* w2) {
  const int npdg = (int)e->pdg_mass.size(), pts = e->gla_pts;
  if (npdg == 0) return e->fail(IS3D_ERR_STATE, "PTB needs the PDG (is3d_set_pdg)");
  std::vector<double> in;
  in.insert(in.end(), e->pdg_mass.begin(), e->pdg_mass.end());
  in.insert(in.end(), e->pdg_degen.begin(), e->pdg_degen.end());
  in.insert(in.end(), e->pdg_sign.begin(), e->pdg_sign.end());
  in.insert(in.end(), r2, r2 + pts);
  in.insert(in.end(), w2, w2 + pts);
  const size_t nterms = (size_t)(kJonahN + 1) * 2 * npdg, nout = 3 * (size_t)kJonahN;
  double* d = dalloc<double>(in.size() + nterms + nout);
  if (!d) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(Jonah table) failed");
  JonahArgs ja{};
  ja.T = e->T_avg; ja.npdg = npdg; ja.pts = pts;
  ja.mass = d; ja.degen = d + npdg; ja.sign = d + 2 * npdg; ja.r2 = d + 3 * npdg; ja.w2 = d + 3 * npdg + pts;
  ja.terms = d + in.size();
  ja.l2 = ja.terms + nterms; ja.z = ja.l2 + kJonahN; ja.bp = ja.z + kJonahN;
  std::vector<double> out(nout);
  hipError_t er = hipMemcpy(d, in.data(), in.size() * sizeof(double), hipMemcpyHostToDevice);
  if (er == hipSuccess) {
    const long nthr = (long)(kJonahN + 1) * npdg;
    hipLaunchKernelGGL(k_jonah_terms, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, 0, ja);
    hipLaunchKernelGGL(k_jonah_sum, dim3((kJonahN + 63) / 64), dim3(64), 0, 0, ja);
    er = hipGetLastError();
  }
  if (er == hipSuccess) er = hipMemcpy(out.data(), ja.l2, nout * sizeof(double), hipMemcpyDeviceToHost);
  dfree(d);
  if (er != hipSuccess) return e->fail(IS3D_ERR_DEVICE, std::string("Jonah table: ") + hipGetErrorString(er));
  e->jl2.assign(out.begin(), out.begin() + kJonahN);
  e->jz.assign(out.begin() + kJonahN, out.begin() + 2 * kJonahN);
  e->jx.assign(out.begin() + 2 * kJonahN, out.end());
  e->bp_max = -1.0;
  for (int i = 0; i < kJonahN; i++) e->bp_max = std::fmax(e->bp_max, e->jx[i]);
  return IS3D_OK;
}

// k_spectra launch shape for this engine's species / grids (shared by the launch and by the {pT cos,
// pT sin} table finalize_tables builds for KJ-padded phi rows)
struct SpectraPlan {
  int KJ, njb, nq, nqmax, tb, ly, t8, tile;
  int ts;                     // F_TS: the F_TB launch with the per-(cell, phi) operands from k_phitab's table
  int by;                     // F_BY: ... with include_baryon (T3 rows)
  int mp, npw;                // F_MP: pT values per workgroup (1 otherwise)
  size_t shmem;
  size_t shmem_fb;            // modified modes: the F_FB launch (8-cell tiles, per-lane y-term rows, no q tables)
};
static SpectraPlan spectra_plan(const is3d_engine* e, bool allow_ts = true) {
  SpectraPlan P{};
  P.npw = 1;
  const int mode = e->p.df_mode, dim = e->p.dimension;
  const int np = e->ncls, nphi = (int)e->phi.size();     // lane species: the integrand classes
  const int npT = (int)e->pT.size();
  const int nk = (dim == 3) ? (int)e->y.size() : 1, nl = (dim == 3) ? 1 : (int)e->eta.size();
  P.nq = nk * nl;
  auto shape = [&](int KJ) {
    P.KJ = KJ;
    P.njb = (nphi + KJ - 1) / KJ;
    // rows (r = q + nq jb) one workgroup's 256 consecutive tasks can span: a contiguous range of at most
    // (kBlock - 1) / np + 2 of the nq njb rows
    P.nqmax = (int)std::min<long>((long)P.nq * P.njb, (kBlock - 1) / np + 2);
    // Grad {PD, T1} table (F_TB, sep_quad_tb_t): exact only without baryon terms (R_SCB = R_SSB = 0:
    // V^mu and alphaB are only packed when include_baryon && include_baryondiff_deltaf (prep_grad_ce), and
    // df_eval leaves c1 = c3 = 0 without baryons); needs phi blocks of fours and at most kTbQ rows per
    // workgroup
    // with include_baryon only as F_TS + F_BY (one phi block of 24 or 32 points: the baryon part of the linear
    // coefficients comes from the table as T3)
    const bool ts_shape = IS3D_TS && IS3D_TS_BY && allow_ts && P.njb == 1 && (KJ == 24 || KJ == 32);
    P.tb = (IS3D_GRAD_TB && (mode == GRAD || (mode == CE && IS3D_CE_TB)) && (!e->p.include_baryon || ts_shape) &&
            KJ % 4 == 0 && P.nqmax <= kTbQ) ? F_TB : 0;
  };
  int kTile = (mode >= PTM) ? IS3D_KTILE_MOD : is3d::kern::kTile;   // spectra_tile<MODE, FLAGS>()
  // k_spectra's LDS layout (kernels.h): record tiles x kRecBufs, per-tile tables x kTabBufs
  // F_TS (kernels.h TS): an F_TB launch with one phi block of 24 or 32 points
  auto ts_ok = [&]() { return IS3D_TS && allow_ts && P.tb && P.njb == 1 && (P.KJ == 24 || P.KJ == 32); };
  bool fb_layout = false;               // sizing the F_FB launch (separable lanes of a modified mode)
  auto lds_bytes = [&](int qrows) {     // qrows = 0: F_LY layout (one y-term row per lane)
    const size_t nphp = (size_t)P.njb * P.KJ, tile = (size_t)kTile;
    // modified launches (kernels.h MODMAIN): the modified lanes' exp table, no {b', Phi} rows (IS3D_MOD_TABLES)
    const bool modmain = mode >= PTM && !fb_layout;
    const size_t etab = modmain ? (size_t)is3d::kModTabN : (size_t)kExpTabN;
    const size_t bprows = (modmain && IS3D_MOD_TABLES) ? 0 : 1;
    if (ts_ok()) {
      // records x 3, trig + {pc, ps}, grid, y-term rows x 2, exp table, T1 rows [tile][qrows][KJ + 2] (+ 1: alignment)
      return sizeof(double) * (3 * tile * NREC + 4 * nphp + (size_t)(nk + 2 * nl) +
                               2 * tile * std::min(qrows, P.nq) * kYRow + kExpTabN + tile * qrows * (P.KJ + 2) + 1 +
                               (IS3D_TS_PF ? 128 : 0));
    }
    // pipelined launches (F_TB, the modified path's 16-cell tiles): 3 record tiles, 2 table buffers
    const bool pipe = IS3D_PIPE && (P.tb || (mode >= PTM && qrows && !P.t8 && !P.ly));
    const size_t rb = pipe ? 3 : 2, tb = pipe ? 2 : 1, qvf = (mode >= PTM || !pipe) ? 2 : 1;
    const size_t w = (size_t)P.npw;     // F_MP: pT blocks of {pc, ps} and of the per-(cell, phi) tables
    return sizeof(double) * (rb * tile * NREC + (2 + 2 * w) * nphp + bprows * tb * 2 * w * tile * nphp + tb * qvf * w * tile * nphp +
                             (size_t)(nk + 2 * nl) +
                             (qrows ? tb * tile * std::min(qrows, P.nq) * kYRow : (size_t)kBlock * kYRowLY) + etab +
                             (P.tb ? 2 * tile * qrows * (P.KJ + 1) + 1 : 0) +
                             (P.tb && mode == CE ? tb * 2 * tile * nphp : 0) +
                             // the per-lane RTA-CE launch's {TE, T2} table (kernels.h PDE)
                             // (+ 1: s_pe starts at the 16-byte-aligned end of the y-term rows)
                             (IS3D_CE_PE && mode == CE && !P.tb && !P.mp && qrows && P.KJ % 4 == 0 ? tb * 2 * tile * nphp + 1 : 0) +
                             (mode >= PTM && qrows ? tile * qrows * (P.KJ + 1) + 1 : 0));
  };
#ifdef IS3D_FORCE_KJ
  shape(IS3D_FORCE_KJ);
#else
  shape(spectra_kj_fill(nphi, (long)np * P.nq));
#endif
  P.ly = 0;
  P.shmem = lds_bytes(P.nqmax);
  // RTA-CE's table launch adds {TE, T2} to the {PD, T1} rows: where that costs the third workgroup per CU
  // (LDS above 160 KB / 3 -- SMASH as 193 integrand classes spans 3 q rows per workgroup: 54.5 KB) the
  // per-lane launch is faster (config 2 RTA-CE 349.7 -> 324.3 ms, profiles/round3_r3h_ab_ce_tb.log; with
  // 444 species, 2 rows, 47.8 KB, the table launch had won 723 -> 676 ms in round 1)
  if (P.tb && mode == CE && 3 * P.shmem > 160 * 1024) {
    P.tb = 0;
    P.shmem = lds_bytes(P.nqmax);
  }
  // the modified path's 16-cell tiles fall back to 8 (F_T8) before giving up the q-row tables
  if (P.shmem > IS3D_LDS_QROW_LIMIT && mode >= PTM && kTile != is3d::kern::kTile) {
    kTile = is3d::kern::kTile;
    P.t8 = F_T8;
    const size_t s8 = lds_bytes(P.nqmax);
    if (s8 <= IS3D_LDS_QROW_LIMIT) P.shmem = s8;
    else { kTile = IS3D_KTILE_MOD; P.t8 = 0; }
  }
  // grids whose q rows do not fit (large y / eta tables with few species; np >= 86 keeps nqmax <= 4) run
  // the F_LY launch (KJ = 8, per-lane y-term rows, no q-row tables) instead of failing: the reference has
  // no grid limit
  if (P.shmem > IS3D_LDS_QROW_LIMIT && !P.tb) {
    shape(8);
    P.tb = 0;
    P.t8 = 0;
    P.ly = F_LY;
    kTile = is3d::kern::kTile;     // spectra_tile<MODE, F_LY | ...>
    P.shmem = lds_bytes(0);
  }
  // F_MP (Grad / RTA-CE, no table launch): when one pT's tasks with a single phi block of KJ >= nphi fill at
  // most half a workgroup (pikp 2+1D: 3 x 24 = 72), a workgroup takes npw = 256 / tasks pT values and every
  // lane a whole phi row -- the lane setup (~4.5 points' work) is paid once per row instead of once per
  // 8-point block; chosen by the same cost model as spectra_kj_fill (lane slots x (KJ + 4.5))
  if (IS3D_MP && mode <= CE && !P.tb && !P.ly && nphi <= 32) {
    const long tpp = (long)np * P.nq;
    const int kjm = nphi <= 24 ? 24 : 32;
    if (tpp * 2 <= kBlock) {
      const long slots = (tpp * P.njb + kBlock - 1) / kBlock * kBlock;
      const double cost_now = (double)slots * (P.KJ + 4.5);
      const int npw = (int)std::min<long>(kBlock / tpp, npT);
      const double cost_mp = (double)kBlock / npw * (kjm + 4.5);
      if (cost_mp < cost_now) {
        SpectraPlan Q = P;
        shape(kjm);
        P.tb = 0;
        P.nqmax = P.nq;
        P.mp = F_MP;
        P.npw = npw;
        const size_t sm = lds_bytes(P.nqmax);
        if (sm <= IS3D_LDS_QROW_LIMIT) P.shmem = sm;
        else P = Q;
      }
    }
  }
  P.ts = ts_ok() ? F_TS : 0;
  P.by = (P.ts && e->p.include_baryon) ? F_BY : 0;
  if (P.ts && kTile != IS3D_KTILE_TS) {     // spectra_tile<MODE, F_TB | F_TS>()
    kTile = IS3D_KTILE_TS;
    P.shmem = lds_bytes(P.nqmax);
    // the F_TS tile's LDS past the limit (a y / eta grid of thousands of nodes): the plan without F_TS
    if (P.shmem > IS3D_LDS_QROW_LIMIT) return spectra_plan(e, false);
  }
  P.tile = kTile;
  if (mode >= PTM) {
    const int t = kTile, ly = P.ly, tb = P.tb, t8 = P.t8;
    kTile = is3d::kern::kTile;
    P.ly = F_LY; P.tb = 0; P.t8 = 0;
    fb_layout = true;
    P.shmem_fb = lds_bytes(0);
    fb_layout = false;
    kTile = t; P.ly = ly; P.tb = tb; P.t8 = t8;
  }
  return P;
}

// PTM's renormalisation n_linear / n_mod (MomentumSpectra.cpp:790-832) is a ratio of two sums that both carry the
// degeneracy as a factor, so it depends on (mass, sign, baryon) alone -- except g = 0, where it is 0 / 0 = NaN and the
// species is skipped.  The renormalisation classes and PTM's integrand classes therefore key on whether g is zero
// (IS3D_PTM_GCLASS 0: SMASH 205 -> 193 PTM lane classes, the same as the other modes; the class representative's g
// cancels to rounding, ~1e-16); IS3D_PTM_GCLASS 1 keys on g itself (round 3 / 4)
#ifndef IS3D_PTM_GCLASS
#define IS3D_PTM_GCLASS 0
#endif
static uint64_t ptm_gkey(double g) {
  return IS3D_PTM_GCLASS ? __builtin_bit_cast(uint64_t, g) : (uint64_t)(g == 0.0 ? 1 : 0);
}

static int finalize_tables(is3d_engine* e) {
  if (!e->have_params) return e->fail(IS3D_ERR_STATE, "is3d_set_params not called");
  if (!e->have_species) return e->fail(IS3D_ERR_STATE, "is3d_set_species not called");
  if (!e->have_grid) return e->fail(IS3D_ERR_STATE, "is3d_set_momentum_grid not called");
  if (!e->have_df) return e->fail(IS3D_ERR_STATE, "is3d_set_df_tables not called");
  const int mode = e->p.df_mode;
  if ((mode == PTM || mode == PTB) && !e->have_gla) return e->fail(IS3D_ERR_STATE, "is3d_set_gauss_laguerre not called");
  if ((mode == PTB || mode == PTMA) && !e->have_pdg) return e->fail(IS3D_ERR_STATE, "is3d_set_pdg not called");
  if (e->p.dimension == 3 && e->y.empty()) return e->fail(IS3D_ERR_ARG, "dimension = 3 needs a y table");
  if (e->p.dimension == 2 && e->eta.empty()) return e->fail(IS3D_ERR_ARG, "dimension = 2 needs an eta table");
  if (!e->tables_dirty) return IS3D_OK;
  HIPCHK(e, hipSetDevice(e->device));
  const int nT = e->nT, nmuB_used = e->p.include_baryon ? e->nmuB : 1;
  // --- delta-f blob: T | muB | tab | 7 x (y, c) | jonah x, l2, l2c, z, zc
  std::vector<double> blob;
  auto put = [&](const double* v, size_t n) { size_t off = blob.size(); blob.insert(blob.end(), v, v + n); return off; };
  const size_t oT = put(e->Tarr.data(), nT);
  const size_t omu = put(e->muBarr.data(), e->nmuB);
  const size_t otab = put(e->tab.data(), e->tab.size());
  size_t osy[NSPL] = {0}, osc[NSPL] = {0};
  const int spl_col[NSPL] = {0, 2, 3, 5, 7, 8, 9};   // c0 c2 c3 F betabulk betaV betapi
  if (!e->p.include_baryon) {
    for (int k = 0; k < NSPL; k++) {
      const double* yv = e->tab.data() + (size_t)spl_col[k] * e->nmuB * nT;   // muB row 0
      std::vector<double> c;
      if (!cspline_coeffs(e->Tarr.data(), yv, nT, c)) return e->fail(IS3D_ERR_ARG, "gsl: x values must be strictly increasing (T table)");
      osy[k] = put(yv, nT);
      osc[k] = put(c.data(), nT);
    }
  }
  size_t ojx = 0, ojl = 0, ojlc = 0, ojz = 0, ojzc = 0;
  int nj = 0;
  if (!e->p.include_baryon && mode == PTB) {
    const double* r2 = e->gla_r.data() + 2 * e->gla_pts;
    const double* w2 = e->gla_w.data() + 2 * e->gla_pts;
    const int rc = device_jonah_table(e, r2, w2);
    if (rc) return rc;
    if (!cspline_coeffs(e->jx.data(), e->jl2.data(), 301, e->jl2c) || !cspline_coeffs(e->jx.data(), e->jz.data(), 301, e->jzc))
      return e->fail(IS3D_ERR_DF_RANGE, "gsl: x values must be strictly increasing (Jonah bulkPi/P table)");
    nj = 301;
    ojx = put(e->jx.data(), 301); ojl = put(e->jl2.data(), 301); ojlc = put(e->jl2c.data(), 301);
    ojz = put(e->jz.data(), 301); ojzc = put(e->jzc.data(), 301);
  }
  dfree(e->d_tables);
  e->d_tables = dalloc<double>(blob.size());
  if (!e->d_tables) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(tables) failed");
  HIPCHK(e, hipMemcpy(e->d_tables, blob.data(), blob.size() * sizeof(double), hipMemcpyHostToDevice));
  DfTables& tb = e->dtb;
  tb.df_mode = mode; tb.include_baryon = e->p.include_baryon;
  tb.nT = nT; tb.nmuB = nmuB_used;
  tb.T = e->d_tables + oT; tb.muB = e->d_tables + omu; tb.tab = e->d_tables + otab;
  tb.T_min = e->Tarr[0]; tb.muB_min = e->muBarr[0];
  tb.dT = std::fabs(e->Tarr[1] - e->Tarr[0]);
  tb.dmuB = e->nmuB > 1 ? std::fabs(e->muBarr[1] - e->muBarr[0]) : 0.0;
  for (int k = 0; k < NSPL; k++) { tb.sy[k] = e->d_tables + osy[k]; tb.sc[k] = e->d_tables + osc[k]; }
  tb.nj = nj; tb.jx = e->d_tables + ojx; tb.jl2 = e->d_tables + ojl; tb.jl2c = e->d_tables + ojlc;
  tb.jz = e->d_tables + ojz; tb.jzc = e->d_tables + ojzc;
  tb.bulk_over_P_max = e->bp_max;
  // tab is laid out [10][nmuB][nT]; with include_baryon = 0 only muB row 0 is used (nmuB_used = 1)
  // but the stride must stay the file's nmuB
  if (!e->p.include_baryon) tb.nmuB = 1;
  // --- constants blob: sorted species, original degeneracy, grids, gla, pdg
  const int np = (int)e->mass.size();
  std::vector<double> cb;
  auto cput = [&](const double* v, size_t n) { size_t off = cb.size(); cb.insert(cb.end(), v, v + n); return off; };
  std::vector<double> sm(np), ss(np), sb(np), sd(np);
  for (int i = 0; i < np; i++) { const int o = e->order[i]; sm[i] = e->mass[o]; ss[i] = e->sign[o]; sb[i] = e->baryon[o]; sd[i] = e->degen[o]; }
  const size_t osm = cput(sm.data(), np), oss = cput(ss.data(), np), osb = cput(sb.data(), np), osd = cput(sd.data(), np);
  const size_t odg = cput(e->degen.data(), np);
  const size_t opt = cput(e->pT.data(), e->pT.size());
  std::vector<double> cph(e->phi.size()), sph(e->phi.size());
  for (size_t j = 0; j < e->phi.size(); j++) { cph[j] = std::cos(e->phi[j]); sph[j] = std::sin(e->phi[j]); }
  const size_t oc = cput(cph.data(), cph.size()), os = cput(sph.data(), sph.size());
  const size_t oy = cput(e->y.data(), e->y.size()), oe = cput(e->eta.data(), e->eta.size()), ow = cput(e->eta_w.data(), e->eta_w.size());
  std::vector<double> pTw(e->pT.size(), 0.0), phiw(e->phi.size(), 0.0);
  if (e->have_weights) { pTw = e->pT_w; phiw = e->phi_w; }
  const size_t opw = cput(pTw.data(), pTw.size()), ophw = cput(phiw.data(), phiw.size());
  // integrand classes of the sorted species (first occurrence order, so the class list stays mass-sorted)
  std::vector<int> scls(np), crep, cmem_off, cmem;
  {
    std::map<std::array<uint64_t, 4>, int> cls;
    for (int i = 0; i < np; i++) {
      const std::array<uint64_t, 4> key{__builtin_bit_cast(uint64_t, sm[i]), __builtin_bit_cast(uint64_t, ss[i]),
                                        __builtin_bit_cast(uint64_t, sb[i]), mode == PTM ? ptm_gkey(sd[i]) : (uint64_t)0};
      int c = (int)crep.size();
      if (e->classes) {
        auto it = cls.find(key);
        if (it == cls.end()) it = cls.emplace(key, c).first;
        c = it->second;
      }
      if (c == (int)crep.size()) crep.push_back(i);
      scls[i] = c;
    }
    const int nc = (int)crep.size();
    cmem_off.assign(nc + 1, 0);
    for (int i = 0; i < np; i++) cmem_off[scls[i] + 1]++;
    for (int c = 0; c < nc; c++) cmem_off[c + 1] += cmem_off[c];
    cmem.resize(np);
    std::vector<int> fill(cmem_off.begin(), cmem_off.end() - 1);
    for (int i = 0; i < np; i++) cmem[fill[scls[i]]++] = i;
    e->ncls = nc;
    e->scls = scls;
  }
  std::vector<double> cm(e->ncls), csn(e->ncls), cby(e->ncls);
  for (int c = 0; c < e->ncls; c++) { cm[c] = sm[crep[c]]; csn[c] = ss[crep[c]]; cby[c] = sb[crep[c]]; }
  const size_t ocm = cput(cm.data(), e->ncls), ocs_ = cput(csn.data(), e->ncls), ocb = cput(cby.data(), e->ncls);
  // {pT cos phi, pT sin phi} per (pT, padded phi slot) for k_spectra's scalar loads (same products as
  // its LDS copy s_cs); 16-byte aligned
  if (cb.size() & 1) cb.push_back(0.0);
  const int kj_cs = spectra_plan(e).KJ;
  const int nphp_cs = (int)((e->phi.size() + kj_cs - 1) / kj_cs) * kj_cs;
  std::vector<double> csv((size_t)e->pT.size() * nphp_cs * 2, 0.0);
  for (size_t i = 0; i < e->pT.size(); i++)
    for (size_t j = 0; j < e->phi.size(); j++) {
      csv[(i * nphp_cs + j) * 2] = e->pT[i] * cph[j];
      csv[(i * nphp_cs + j) * 2 + 1] = e->pT[i] * sph[j];
    }
  const size_t ocs = cput(csv.data(), csv.size());
  const size_t og = cput(e->gla_r.data(), e->gla_r.size());
  cput(e->gla_w.data(), e->gla_w.size());
  const size_t opd = cput(e->pdg_mass.data(), e->pdg_mass.size());
  cput(e->pdg_sign.data(), e->pdg_sign.size());
  cput(e->pdg_degen.data(), e->pdg_degen.size());
  // PTMA Newton solve / famod coefficients: the reference sums its first min(320, N) PDG hadrons
  // (MomentumSpectra.cpp:1295); the integrands depend on a hadron's (mass, sign) only, times its
  // degeneracy, so hadrons with identical (mass, sign) are merged with summed degeneracies (SMASH:
  // 320 -> 92, UrQMD: 320 -> 83; first-occurrence order).  Only the FP summation order changes, as it
  // already does in the lane-strided sums.  Checked on the breakdown-heavy chain (bulk x10, one chain,
  // tests/test_gpu_configs.py::test_modified_fallback_launch): the merged GPU solve and the unmerged
  // oracle take the same 894 Newton steps and agree to 3e-13; tests/test_kernel_math_cpu.py compares
  // merged and per-hadron sums of the same device math directly (cf_emulator variant bit 8).
  std::vector<double> am, as, ag;
  {
    const int nh = std::min(320, (int)e->pdg_mass.size());
    for (int i = 0; i < nh; i++) {
      int k = -1;
      if (IS3D_ANISO_MERGE)
        for (size_t u = 0; u < am.size(); u++)
          if (am[u] == e->pdg_mass[i] && as[u] == e->pdg_sign[i]) { k = (int)u; break; }
      if (k < 0) { am.push_back(e->pdg_mass[i]); as.push_back(e->pdg_sign[i]); ag.push_back(e->pdg_degen[i]); }
      else ag[k] += e->pdg_degen[i];
    }
    if (am.empty()) { am.push_back(0.0); as.push_back(0.0); ag.push_back(0.0); }
  }
  e->n_aniso_h = e->pdg_mass.empty() ? 0 : (int)am.size();
  const size_t oah = cput(am.data(), am.size());
  cput(as.data(), as.size());
  cput(ag.data(), ag.size());
  std::vector<int> rcls(np), rrep;
  {
    std::map<std::array<uint64_t, 4>, int> cls;
    for (int i = 0; i < np; i++) {
      const std::array<uint64_t, 4> key{__builtin_bit_cast(uint64_t, sm[i]), __builtin_bit_cast(uint64_t, ss[i]),
                                        ptm_gkey(sd[i]), __builtin_bit_cast(uint64_t, sb[i])};
      auto it = cls.find(key);
      if (it == cls.end()) { it = cls.emplace(key, (int)rrep.size()).first; rrep.push_back(i); }
      rcls[i] = it->second;
    }
  }
  e->nrcls = (int)rrep.size();
  const int nc = e->ncls;
  std::vector<int> crcls(nc);
  for (int c = 0; c < nc; c++) crcls[c] = rcls[crep[c]];
  // ints after the doubles: sorig[np] | rcls[np] | rrep[np] | crcls[nc] | cmem_off[nc + 1] | cmem[np] | scls[np]
  std::vector<int> ib;
  for (int i = 0; i < np; i++) ib.push_back(e->order[i]);
  ib.insert(ib.end(), rcls.begin(), rcls.end());
  rrep.resize(np, 0);
  ib.insert(ib.end(), rrep.begin(), rrep.end());
  ib.insert(ib.end(), crcls.begin(), crcls.end());
  ib.insert(ib.end(), cmem_off.begin(), cmem_off.end());
  ib.insert(ib.end(), cmem.begin(), cmem.end());
  ib.insert(ib.end(), scls.begin(), scls.end());
  dfree(e->d_const);
  e->d_const = dalloc<double>(cb.size() + (ib.size() + 1) / 2);
  if (!e->d_const) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(constants) failed");
  HIPCHK(e, hipMemcpy(e->d_const, cb.data(), cb.size() * sizeof(double), hipMemcpyHostToDevice));
  int* const di = (int*)(e->d_const + cb.size());
  HIPCHK(e, hipMemcpy(di, ib.data(), ib.size() * sizeof(int), hipMemcpyHostToDevice));
  e->d_sorig = di;
  e->d_rcls = di + np;
  e->d_rrep = di + 2 * (size_t)np;
  e->d_crcls = di + 3 * (size_t)np;
  e->d_cmem_off = e->d_crcls + nc;
  e->d_cmem = e->d_cmem_off + nc + 1;
  e->d_scls = e->d_cmem + np;
  e->d_cmass = e->d_const + ocm; e->d_csign = e->d_const + ocs_; e->d_cbaryon = e->d_const + ocb;
  e->d_smass = e->d_const + osm; e->d_ssign = e->d_const + oss; e->d_sbaryon = e->d_const + osb; e->d_sdegen = e->d_const + osd;
  e->d_degen_orig = e->d_const + odg; e->d_pT = e->d_const + opt; e->d_cphi = e->d_const + oc; e->d_sphi = e->d_const + os;
  e->d_y = e->d_const + oy; e->d_eta = e->d_const + oe; e->d_etaw = e->d_const + ow;
  e->d_gla = e->d_const + og; e->d_pdg = e->d_const + opd; e->d_aniso_h = e->d_const + oah;
  e->d_pTw = e->d_const + opw; e->d_phiw = e->d_const + ophw;
  e->d_csg = e->d_const + ocs;
  e->tables_dirty = false;
  return IS3D_OK;
}

extern "C" int is3d_set_surface(is3d_engine* e, long n, const is3d_surface* s) {
  if (e && e->grp) return is3d::group_set_surface(e->grp, n, s);
  if (!e || !s || n < 0) return e ? e->fail(IS3D_ERR_ARG, "bad surface") : IS3D_ERR_ARG;
  HIPCHK(e, hipSetDevice(e->device));
  const double* fields[NSURF] = {s->tau, s->x, s->y, s->eta, s->dat, s->dax, s->day, s->dan, s->ux, s->uy, s->un,
                                 s->E, s->T, s->P, s->pixx, s->pixy, s->pixn, s->piyy, s->piyn, s->bulkPi,
                                 s->muB, s->nB, s->Vx, s->Vy, s->Vn};
  for (int f = 0; f < S_MUB; f++)
    if (!fields[f] && n > 0) return e->fail(IS3D_ERR_ARG, "surface field missing");
  // (reallocated when too small, or more than twice the size: a device group's cost prepass uploads the whole
  // surface to shard 0 before its own window)
  if (!e->surf_owned || e->surf_cap < n || e->surf_cap > 2 * n + 4096) {
    if (e->surf_owned) dfree(e->d_surf);
    e->d_surf = dalloc<double>((size_t)NSURF * std::max(n, 1L));
    if (!e->d_surf) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(surface) failed");
    e->surf_owned = true;
    e->surf_cap = n;
  }
  e->ncell = n;
  e->win_lo = e->win_hi = -1;
  e->chain_q0 = e->chain_q1 = -1;
  if (n == 0) return IS3D_OK;
  for (int f = 0; f < NSURF; f++) {
    double* dst = e->d_surf + (size_t)f * n;
    if (fields[f]) HIPCHK(e, hipMemcpy(dst, fields[f], n * sizeof(double), hipMemcpyHostToDevice));
    else HIPCHK(e, hipMemset(dst, 0, n * sizeof(double)));
  }
  return IS3D_OK;
}

extern "C" int is3d_set_surface_device(is3d_engine* e, long n, const double* dev_fields) {
  if (e && e->grp) return is3d::group_set_surface_device(e->grp, n, dev_fields);
  if (!e || n < 0 || (!dev_fields && n > 0)) return e ? e->fail(IS3D_ERR_ARG, "bad device surface") : IS3D_ERR_ARG;
  if (e->surf_owned) dfree(e->d_surf);
  e->surf_owned = false;
  e->surf_cap = 0;
  e->d_surf = const_cast<double*>(dev_fields);
  e->ncell = n;
  e->win_lo = e->win_hi = -1;
  e->chain_q0 = e->chain_q1 = -1;
  return IS3D_OK;
}

extern "C" int is3d_internal_copy_surface(is3d_engine* e, long n, const double* src, long src_n, int src_device, long lo) {
  if (!e || e->grp || n < 0 || lo < 0 || lo + n > src_n || (!src && n > 0)) return e ? e->fail(IS3D_ERR_ARG, "bad surface copy") : IS3D_ERR_ARG;
  HIPCHK(e, hipSetDevice(e->device));
  // (reallocated when too small, or more than twice the size: a device group's cost prepass uploads the whole
  // surface to shard 0 before its own window)
  if (!e->surf_owned || e->surf_cap < n || e->surf_cap > 2 * n + 4096) {
    if (e->surf_owned) dfree(e->d_surf);
    e->d_surf = dalloc<double>((size_t)NSURF * std::max(n, 1L));
    if (!e->d_surf) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(surface) failed");
    e->surf_owned = true;
    e->surf_cap = n;
  }
  e->ncell = n;
  e->win_lo = e->win_hi = -1;
  e->chain_q0 = e->chain_q1 = -1;
  for (int f = 0; f < NSURF && n > 0; f++)
    HIPCHK(e, hipMemcpyPeer(e->d_surf + (size_t)f * n, e->device, src + (size_t)f * src_n + lo, src_device, n * sizeof(double)));
  return IS3D_OK;
}

extern "C" long is3d_output_size(const is3d_engine* e) {
  if (e && e->grp) return is3d::group_output_size(e->grp);
  if (!e || !e->have_species || !e->have_grid || !e->have_params) return -1;
  const long ny = (e->p.dimension == 3) ? (long)e->y.size() : 1;
  return (long)e->mass.size() * (long)e->pT.size() * (long)e->phi.size() * ny;
}

template <class T>
static bool ensure(T*& p, long& cap, long need) {
  if (cap >= need && p) return true;
  dfree(p);
  p = dalloc<T>((size_t)std::max(need, 1L));
  cap = p ? need : 0;
  return p != nullptr;
}

static PrepConsts make_consts(const is3d_engine* e) {
  PrepConsts k{};
  k.operation = 1;
  k.df_mode = e->p.df_mode; k.dim = e->p.dimension; k.include_baryon = e->p.include_baryon;
  k.include_bulk = e->p.include_bulk_deltaf; k.include_shear = e->p.include_shear_deltaf;
  k.include_diff = e->p.include_baryondiff_deltaf;
  k.deta_min = e->p.deta_min; k.mass_pion0 = e->p.mass_pion0;
  k.gla_pts = e->gla_pts;
  if (e->have_gla) {
    k.gla_r1 = e->d_gla + 1 * e->gla_pts; k.gla_r2 = e->d_gla + 2 * e->gla_pts;
    const double* w = e->d_gla + (size_t)e->gla_alpha * e->gla_pts;
    k.gla_w1 = w + 1 * e->gla_pts; k.gla_w2 = w + 2 * e->gla_pts;
  }
  k.two_pi2_hbarC3 = 2.0 * std::pow(M_PI, 2) * std::pow(kHbarC, 3);
  k.pT_max = 0.0; k.b_max = 0.0;
  for (double v : e->pT) k.pT_max = std::max(k.pT_max, std::fabs(v));
  for (double v : e->baryon) k.b_max = std::max(k.b_max, std::fabs(v));
  return k;
}

// A launch in stages: launch_begin (prepass up to PTMA's warm-start chains), chain_pass x npass + chain_end (the
// chains), launch_end (PTMA C/B matrices, PTM renormalisation, the integral, the reduction).  is3d_launch runs them
// back to back; a device group whose shards solve their own ranges of the chains (group.hip) interleaves the
// shards' passes with the boundary hand-offs between them.
static int launch_begin(is3d_engine* e, double* dev_out, void* stream, long q0, long q1, int has_pred) {
  int rc = finalize_tables(e);
  if (rc) return rc;
  if (!dev_out) return e->fail(IS3D_ERR_ARG, "null output buffer");
  HIPCHK(e, hipSetDevice(e->device));
  LaunchCtx& L = e->lc;
  L = LaunchCtx{};
  hipStream_t st = (hipStream_t)stream;
  L.st = st; L.dev_out = dev_out;
  const long n = e->ncell;
  const int mode = e->p.df_mode;
  const long outsize = is3d_output_size(e);
  // cell window (group shards holding the whole surface): k_spectra integrates [wlo, whi); the prepass covers
  // the window too, except for PTMA's warm-start chains, which walk every cell (MomentumSpectra.cpp:1308-1364) --
  // or, when a device group splits the chains (q1 >= 0), the cells of this shard's positions, which are its window
  const long wlo = e->win_hi >= 0 ? e->win_lo : 0, whi = e->win_hi >= 0 ? e->win_hi : n, nw = whi - wlo;
  const bool chained = mode == PTMA && e->p.famod_chains > 0;
  const bool split_chain = chained && q1 >= 0;
  const long p0 = chained && !split_chain ? 0 : wlo, p1 = chained && !split_chain ? n : whi;
  L.wlo = wlo; L.whi = whi; L.nw = nw; L.p0 = p0; L.p1 = p1; L.chained = chained;
  e->st = is3d_stats{};
  e->st.cells = nw;
  HIPCHK(e, hipMemsetAsync(e->d_err, 0, sizeof(int), st));
  HIPCHK(e, hipMemsetAsync(e->d_cnt, 0, 8 * sizeof(unsigned long long), st));
  HIPCHK(e, hipEventRecord(e->ev[0], st));
  if (nw == 0) {
    L.empty = true;
    HIPCHK(e, hipMemsetAsync(dev_out, 0, outsize * sizeof(double), st));
    return IS3D_OK;
  }
  if (!ensure(e->d_rec, e->rec_cap, (long)NREC * n)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(records) failed");
  if (!ensure(e->d_aux, e->aux_cap, 9L * n)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(aux) failed");
  if (mode == PTMA && !ensure(e->d_sol, e->sol_cap, 6L * n)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(sol) failed");
  PrepArgs& pa = L.pa;
  pa.k = make_consts(e); pa.tb = e->dtb; pa.surf = e->d_surf; pa.rec = e->d_rec; pa.aux = e->d_aux; pa.n = n;
  pa.c0 = p0; pa.c1 = p1;
  pa.err = e->d_err; pa.cnt = e->d_cnt;
  const dim3 g1((unsigned)std::max(1L, (p1 - p0 + 255) / 256)), b1(256);
  switch (mode) {
    case GRAD: hipLaunchKernelGGL(k_prep<GRAD>, g1, b1, 0, st, pa); break;
    case CE: hipLaunchKernelGGL(k_prep<CE>, g1, b1, 0, st, pa); break;
    case PTM: hipLaunchKernelGGL(k_prep<PTM>, g1, b1, 0, st, pa); break;
    case PTB: hipLaunchKernelGGL(k_prep<PTB>, g1, b1, 0, st, pa); break;
    default: hipLaunchKernelGGL(k_prep<PTMA>, g1, b1, 0, st, pa); break;
  }
  HIPCHK(e, hipGetLastError());
  if (mode == PTMA) {
    AnisoArgs aa{};
    aa.rec = e->d_rec; aa.ain = e->d_aux; aa.sol = e->d_sol; aa.stride = n;
    aa.c0 = p0; aa.n = p1 - p0;
    aa.chains = chained ? std::min<long>(e->p.famod_chains, n) : std::max(1L, p1 - p0);
    const int nh = e->n_aniso_h;
    aa.h = Hadrons{nh, e->d_aniso_h, e->d_aniso_h + nh, e->d_aniso_h + 2 * nh};
    aa.fp2 = 4.0 * std::pow(M_PI, 2) * std::pow(kHbarC, 3);
    aa.cnt = e->d_cnt;
    if (!chained) {
      hipLaunchKernelGGL(k_aniso, dim3((unsigned)aa.chains), dim3(64), 0, st, aa);
      HIPCHK(e, hipGetLastError());
    } else {
      // warm-start chains in parallel segments (k_chain_pass): ~16k segments of this engine's positions keep the
      // GPU full
      ChainArgs& ca = L.ca;
      ca.rec = e->d_rec; ca.ain = e->d_aux; ca.sol = e->d_sol; ca.n = n; ca.C = aa.chains; ca.h = aa.h; ca.fp2 = aa.fp2;
      const long P = (n + ca.C - 1) / ca.C;
      ca.q0 = split_chain ? q0 : 0;
      ca.q1 = split_chain ? std::min(q1, P) : P;
      ca.has_pred = split_chain && has_pred && ca.q0 > 0;
      const long npos = std::max(1L, ca.q1 - ca.q0);
      // ~IS3D_CHAIN_SLOTS segments of at least IS3D_CHAIN_L positions (sized to the GPU's resident k_chain_pass
      // wavefronts instead -- 2048, L = 49 at 10^5 cells -- measured the same: profiles/round4_r4b_ab_newton.log)
      long slots = IS3D_CHAIN_SLOTS;
      if (const char* v = std::getenv("IS3D_CHAIN_SLOTS")) slots = std::max(1L, std::atol(v));   // A/B knob
      const long spc_max = std::max(1L, slots / ca.C);
      ca.L = std::max((long)IS3D_CHAIN_L, (npos + spc_max - 1) / spc_max);
      ca.nspc = (npos + ca.L - 1) / ca.L;
      ca.npass = kChainPasses;
      if (const char* v = std::getenv("IS3D_CHAIN_PASSES")) ca.npass = std::max(1, std::min(kChainPasses, std::atoi(v)));
      const long nseg = ca.C * ca.nspc, bw = 4 * ca.C + 1;
      const long need = 4 * n + (n + 1) / 2 + 12 * nseg + kChainPasses + 2 * kBndSlots * bw;
      if (!ensure(e->d_chain, e->chain_cap, need)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(chain state) failed");
      ca.sta = e->d_chain; ca.info = (int*)(e->d_chain + 4 * n);
      ca.send = e->d_chain + 4 * n + (n + 1) / 2; ca.sstart = ca.send + 8 * nseg;
      ca.changed = (int*)(ca.sstart + 4 * nseg);
      ca.bin = ca.sstart + 4 * nseg + kChainPasses;
      ca.bout = ca.bin + kBndSlots * bw;
      HIPCHK(e, hipMemsetAsync(ca.changed, 0, kChainPasses * sizeof(int), st));
    }
  }
  return IS3D_OK;
}

static int chain_pass(is3d_engine* e, int pass) {
  LaunchCtx& L = e->lc;
  if (L.empty || !L.chained) return IS3D_OK;
  HIPCHK(e, hipSetDevice(e->device));
  hipLaunchKernelGGL(k_chain_pass, dim3((unsigned)(L.ca.C * L.ca.nspc)), dim3(64 * IS3D_CHAIN_W), 0, L.st, L.ca, pass);
  HIPCHK(e, hipGetLastError());
  return IS3D_OK;
}

static int chain_end(is3d_engine* e) {
  LaunchCtx& L = e->lc;
  if (L.empty || !L.chained) return IS3D_OK;
  HIPCHK(e, hipSetDevice(e->device));
  const long c_lo = L.ca.q0 * L.ca.C, c_hi = std::min(e->ncell, L.ca.q1 * L.ca.C);
  hipLaunchKernelGGL(k_chain_finish, dim3(1), dim3(64 * IS3D_CHAIN_W), 0, L.st, L.ca);
  hipLaunchKernelGGL(k_chain_count, dim3((unsigned)std::min(1024L, std::max(1L, (c_hi - c_lo + 255) / 256))), dim3(256), 0,
                     L.st, (const double*)e->d_rec, (const int*)L.ca.info, c_lo, c_hi, e->d_cnt);
  HIPCHK(e, hipGetLastError());
  return IS3D_OK;
}

// Cell splits and slab geometry of one k_spectra plan over a launch window of nw cells.
struct IntegralPlan {
  SpectraPlan P;
  long ntask = 0, bx = 0, wgs = 0, nsplit = 0, cps = 0, sstride = 0, nsplit_fb = 0;
  // F_TS table chunks: spc splits per chunk, nchunk chunks; fold: each chunk's slabs are folded into one accumulator
  // slab as soon as the chunk is integrated (3+1D, several chunks), so the slabs take 1 + 2 spc output sizes of HBM
  // instead of nsplit (config 4: 947 -> 67 slabs, 47 -> 3.4 GB)
  long spc = 0, nchunk = 0, rw = 0;
  bool fold = false;
  long slabs() const { return fold ? 1 + 2 * spc : nsplit + nsplit_fb; }
};

#ifndef IS3D_SLAB_FOLD
#define IS3D_SLAB_FOLD 1
#endif

// F_TS chunking of plan I over nw cells: tables of the whole window up to phitab_one bytes in one chunk, larger ones in
// chunks of whole cell splits of about phitab_chunk bytes; both within half the device's free memory (plus the table
// buffers this engine already holds)
static void ts_chunking(is3d_engine* e, IntegralPlan& I) {
  const int npT = (int)e->pT.size();
  I.rw = phitab_row(e->p.df_mode, I.P.KJ, I.P.by != 0);
  const long per_split = I.cps * (long)npT * I.rw;
  const long whole = per_split * I.nsplit * 8;          // bytes of the whole surface's rows
  long one = e->phitab_one, chunk = e->phitab_chunk;
  {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot > 0) {
      const long avail = (long)(fr / 2) + (e->phtab_cap + e->phtab2_cap) * (long)sizeof(double);
      one = std::min(one, avail);
      chunk = std::max(8L * per_split, std::min(chunk, avail / 2));
    }
  }
  const long budget = whole <= one ? whole : chunk;
  I.spc = std::max(1L, std::min(I.nsplit, budget / 8 / per_split));
  I.nchunk = (I.nsplit + I.spc - 1) / I.spc;
  I.fold = IS3D_SLAB_FOLD && I.nchunk > 1 && e->p.dimension == 3 && I.nsplit_fb == 0;
}

static int integral_plan(is3d_engine* e, const SpectraPlan& P, long nw, IntegralPlan& I, long cap_slabs = 0) {
  const int dim = e->p.dimension, mode = e->p.df_mode;
  const int npT = (int)e->pT.size();
  const int nk = (dim == 3) ? (int)e->y.size() : 1, nl = (dim == 3) ? 1 : (int)e->eta.size();
  const int KJ = P.KJ, njb = P.njb;
  if (!spectra_kj_supported(KJ)) return e->fail(IS3D_ERR_ARG, "internal: no k_spectra instantiation for this phi block");
  if (P.shmem > 160 * 1024) return e->fail(IS3D_ERR_ARG, "momentum grid too large for the LDS tile (phi table)");
  const int nc = e->ncls;      // lane species: one per integrand class (the reduction writes the members)
  const long ntask = (long)nc * nk * nl * njb;
  const long bx = (ntask + kBlock - 1) / kBlock;            // lane groups per pT (F_MP: 1, ntask <= 128)
  if (!P.ly) {
    // k_spectra's LDS row tables hold nqmax rows per cell; a lane group spanning more would compute nothing
    // (its slab is NaN-filled, rows_ok), so refuse the launch here instead of returning NaN spectra
    for (long g = 0; g < bx; g++) {
      const long t0 = g * kBlock, t1 = std::min(ntask, t0 + kBlock) - 1;
      if (t1 / nc - t0 / nc + 1 > P.nqmax)
        return e->fail(IS3D_ERR_ARG, "internal: k_spectra lane group spans more q rows than the LDS plan");
    }
  }
  // workgroups per cell split: lane groups x pT values, or F_MP's pT groups of npw
  const long npg = P.mp ? (npT + P.npw - 1) / P.npw : npT;
  const long wgs = bx * npg;
  // cell splits: enough workgroups to fill the chip (>= 8k), and each split's records small enough
  // (~0.5 MB, with the PTM renormalisation rows 2 MB) to stay in one XCD's 4 MB L2 while that XCD's workgroups stream them; a multiple of 8
  // so every XCD owns whole splits; at most IS3D_MAX_SPLITS slabs (each one output-sized)
  const long kTile = P.tile;                              // cells per tile of this mode's k_spectra
  const long max_split = std::max(1L, (nw + kTile - 1) / kTile);
  // (F_MP launches aim for 2k: their 2+1D slabs hold every eta node, and k_reduce_wave's reads across 1k
  // splits cost config 1's shape 0.5 ms of a 4.7 ms pass -- Grad 4.7 -> 4.2 ms, RTA-CE 5.4 -> 5.0 ms with 2k,
  // while the F_LY launch of the modified modes lost 14% with it: profiles/round3_r3p_ab_fill.log)
  const long by_fill = ((P.mp ? IS3D_FILL_WGS_MP : IS3D_FILL_WGS) + wgs - 1) / wgs;
  const long by_l2 = ((long)NREC * 8 * nw + e->split_bytes - 1) / e->split_bytes;
  const long sstride = (long)npT * bx * KJ * kBlock;
  // slab memory: the tuning cap, and at most half of the device's total memory -- deterministic inputs only, since
  // the split count sets the summation order (free memory changes from launch to launch with other engines, ranks
  // and torch's cache; it decides only the F_TS chunking and folding below, which leave the bits unchanged)
  long slab_budget = e->slab_bytes;
  {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && tot > 0) slab_budget = std::min(slab_budget, (long)(tot / 2));
  }
  long max_slabs = std::max(8L, std::min(e->max_splits, (slab_budget / 8) / std::max(1L, sstride)));
  if (cap_slabs > 0) max_slabs = std::min(max_slabs, cap_slabs);
  long nsplit = std::max(by_fill, std::min(by_l2, max_slabs));
  if (nsplit >= 8) nsplit = (nsplit + 7) / 8 * 8;
  nsplit = std::max(1L, std::min(nsplit, max_split));
  long cps = std::max(1L, (nw + nsplit - 1) / nsplit);
  cps = ((cps + kTile - 1) / kTile) * kTile;
  nsplit = std::max(1L, (nw + cps - 1) / cps);
  I.P = P; I.ntask = ntask; I.bx = bx; I.wgs = wgs; I.nsplit = nsplit; I.cps = cps; I.sstride = sstride;
  // modified modes: the F_FB launch (separable-fallback lanes, cells listed by k_fbcount / k_fbwrite) writes its own
  // nsplit_fb slabs after the main ones; k_reduce sums both
  I.nsplit_fb = (mode >= PTM) ? std::max(1L, std::min(nsplit, 8L)) : 0;
  if (P.ts) ts_chunking(e, I);
  return IS3D_OK;
}

// the integral of one plan over the launch window (records rec_w, nw cells) into the slabs; gate: launch_end's
// device-side choice between two plans (kernels.h gate_closed), nullptr = unconditional
static int enqueue_spectra(is3d_engine* e, const IntegralPlan& I, const double* rec_w, long nw, hipStream_t st,
                           const unsigned long long* gate, int want) {
  const SpectraPlan& P = I.P;
  const int mode = e->p.df_mode, dim = e->p.dimension;
  const int npT = (int)e->pT.size(), nphi = (int)e->phi.size();
  const int ny_out = (dim == 3) ? (int)e->y.size() : 1;
  const int nk = ny_out, nl = (dim == 3) ? 1 : (int)e->eta.size();
  const int KJ = P.KJ, njb = P.njb, nc = e->ncls;
  const long nsplit = I.nsplit, cps = I.cps, wgs = I.wgs;
  if (mode >= PTM) {
    if (!ensure(e->d_fb, e->fb_cap, nw + 1 + kFbBlocks)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(fallback list) failed");
    enqueue_fbscan(rec_w, nw, e->d_fb, st);
    HIPCHK(e, hipGetLastError());
  }
  SpecArgs sa{};
  sa.err = e->d_err;
  sa.rec = rec_w; sa.n = nw; sa.renorm = e->d_renorm; sa.rcls = e->d_crcls; sa.nrcls = e->nrcls; sa.slab = e->d_slab;
  sa.outsize = is3d_output_size(e);
  sa.smass = e->d_cmass; sa.ssign = e->d_csign; sa.sbaryon = e->d_cbaryon; sa.sorig = e->d_sorig;
  sa.csg = e->d_csg;
  sa.pT = e->d_pT; sa.cphi = e->d_cphi; sa.sphi = e->d_sphi; sa.yv = e->d_y; sa.etav = e->d_eta; sa.etaw = e->d_etaw;
  sa.npart = nc; sa.npT = npT; sa.nphi = nphi; sa.ny_out = ny_out; sa.nk = nk; sa.nl = nl; sa.nq = nk * nl; sa.njb = njb;
  sa.nqmax = P.nqmax;
  sa.ntask = I.ntask; sa.cells_per_split = cps; sa.nbx = (int)I.bx; sa.nsplit = (int)nsplit; sa.sstride = I.sstride;
  sa.npw = P.npw;
  sa.regulate = e->p.regulate_deltaf; sa.outflow = e->p.outflow; sa.dim = dim; sa.op = 1;
  sa.gate = gate; sa.gate_want = want;
  const size_t shmem = P.shmem;
  const int tb = P.tb | P.ly | P.t8 | P.mp | P.ts | P.by;
  const int kflags = (e->p.regulate_deltaf ? F_REG : 0) | (e->p.outflow ? F_OUT : 0) | tb;
  if (P.ts) {
    // F_TS: k_phitab writes the per-(cell, pT, phi) rows of a chunk of whole cell splits (at most
    // phitab_chunk bytes, is3d_set_tuning), then k_spectra integrates that chunk's splits; one chunk at config 2
    // (3.7 GB).  Several chunks (config 4: 61 GB of rows) alternate between the launch stream and a side stream
    // with a table buffer each, so the next chunk's k_phitab and the first workgroups of its k_spectra fill the
    // CUs the previous launch's last workgroups leave idle (config 4: 11 chunks ran 2811 ms back to back, one
    // 61 GB chunk 2739 ms)
    const long rw = I.rw, spc = I.spc, nchunk = I.nchunk;
    const long phn = spc * cps;
    e->last_nchunk = nchunk;
    if (!ensure(e->d_phtab, e->phtab_cap, phn * npT * rw)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(phi tables) failed");
    if (nchunk > 1) {
      if (!ensure(e->d_phtab2, e->phtab2_cap, phn * npT * rw)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(phi tables) failed");
      if (!e->side) HIPCHK(e, hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking));
      if (!e->fork) HIPCHK(e, hipEventCreateWithFlags(&e->fork, hipEventDisableTiming));
      if (!e->join) HIPCHK(e, hipEventCreateWithFlags(&e->join, hipEventDisableTiming));
      HIPCHK(e, hipEventRecord(e->fork, st));
      HIPCHK(e, hipStreamWaitEvent(e->side, e->fork, 0));
    }
    if (I.fold) {
      if (!e->fold_st) HIPCHK(e, hipStreamCreateWithFlags(&e->fold_st, hipStreamNonBlocking));
      for (auto* v : {&e->ev_spec[0], &e->ev_spec[1], &e->ev_fold[0], &e->ev_fold[1], &e->fold_join})
        if (!*v) HIPCHK(e, hipEventCreateWithFlags(v, hipEventDisableTiming));
      HIPCHK(e, hipStreamWaitEvent(e->fold_st, e->fork, 0));
    }
    // folded: slab 0 is the accumulator, chunk ic's splits go to buffer ic & 1 (slabs 1 + (ic & 1) spc ...)
    const int fgrid = (int)std::min(4096L, std::max(1L, (I.sstride + 255) / 256));
    for (long ic = 0; ic < nchunk; ic++) {
      const long s0 = ic * spc, ns = std::min(spc, nsplit - s0);
      const long c0 = s0 * cps, ncc = std::min(nw, (s0 + ns) * cps) - c0;
      hipStream_t cs = (ic & 1) ? e->side : st;
      double* tab = (ic & 1) ? e->d_phtab2 : e->d_phtab;
      PhiTabArgs ta{};
      ta.rec = rec_w; ta.c0 = c0; ta.nc = ncc; ta.pT = e->d_pT; ta.cphi = e->d_cphi; ta.sphi = e->d_sphi;
      ta.npT = npT; ta.nphi = nphi; ta.nphp = KJ; ta.tab = tab; ta.phn = phn; ta.by = P.by != 0;
      ta.gate = gate; ta.gate_want = want;
      SpecArgs sc = sa;
      sc.split0 = (int)s0; sc.nsplit = (int)ns; sc.phtab = tab; sc.phn = phn; sc.phc0 = c0; sc.phrow = (int)rw;
      double* buf = e->d_slab + (1 + (ic & 1) * spc) * I.sstride;
      if (I.fold) { sc.slab = buf; sc.slab0 = (int)s0; }
      const dim3 grid((unsigned)(wgs * ns));
      if (mode == GRAD) launch_phitab<GRAD>(cs, ta);
      else launch_phitab<CE>(cs, ta);
      // a folded chunk reusing slab buffer ic & 1 waits for the fold of chunk ic - 2, which emptied it
      if (I.fold && ic >= 2) HIPCHK(e, hipStreamWaitEvent(cs, e->ev_fold[ic & 1], 0));
      if (mode == GRAD) launch_spectra<GRAD>(grid, shmem, cs, sc, kflags, KJ);
      else launch_spectra<CE>(grid, shmem, cs, sc, kflags, KJ);
      HIPCHK(e, hipGetLastError());
      if (I.fold) {
        HIPCHK(e, hipEventRecord(e->ev_spec[ic & 1], cs));
        HIPCHK(e, hipStreamWaitEvent(e->fold_st, e->ev_spec[ic & 1], 0));
        hipLaunchKernelGGL(k_fold, dim3((unsigned)fgrid), dim3(256), 0, e->fold_st, e->d_slab, (const double*)buf,
                           I.sstride, (int)ns, ic == 0 ? 1 : 0, gate, want);
        HIPCHK(e, hipGetLastError());
        HIPCHK(e, hipEventRecord(e->ev_fold[ic & 1], e->fold_st));
      }
    }
    if (nchunk > 1) {
      HIPCHK(e, hipEventRecord(e->join, e->side));
      HIPCHK(e, hipStreamWaitEvent(st, e->join, 0));
    }
    if (I.fold) {
      HIPCHK(e, hipEventRecord(e->fold_join, e->fold_st));
      HIPCHK(e, hipStreamWaitEvent(st, e->fold_join, 0));
    }
  } else {
    const dim3 grid((unsigned)(wgs * nsplit));
    switch (mode) {
      case GRAD: launch_spectra<GRAD>(grid, shmem, st, sa, kflags, KJ); break;
      case CE: launch_spectra<CE>(grid, shmem, st, sa, kflags, KJ); break;
      case PTM: launch_spectra<PTM>(grid, shmem, st, sa, kflags, KJ); break;
      case PTB: launch_spectra<PTB>(grid, shmem, st, sa, kflags, KJ); break;
      default: launch_spectra<PTMA>(grid, shmem, st, sa, kflags, KJ); break;
    }
  }
  HIPCHK(e, hipGetLastError());
  if (mode >= PTM) {
    SpecArgs fa = sa;
    fa.slab = e->d_slab + nsplit * I.sstride; fa.nsplit = (int)I.nsplit_fb; fa.cells_per_split = 0;
    fa.fbcells = e->d_fb + 1; fa.fbcount = e->d_fb;
    const int fflags = (e->p.regulate_deltaf ? F_REG : 0) | (e->p.outflow ? F_OUT : 0) | F_FB;
    const dim3 gfb((unsigned)(I.bx * npT * I.nsplit_fb));
    switch (mode) {
      case PTM: launch_spectra<PTM>(gfb, P.shmem_fb, st, fa, fflags, KJ); break;
      case PTB: launch_spectra<PTB>(gfb, P.shmem_fb, st, fa, fflags, KJ); break;
      default: launch_spectra<PTMA>(gfb, P.shmem_fb, st, fa, fflags, KJ); break;
    }
    HIPCHK(e, hipGetLastError());
  }
  return IS3D_OK;
}

// sum of one plan's slabs into the reference-layout output (k_reduce / k_reduce_wave), gated as enqueue_spectra
static int enqueue_reduce(is3d_engine* e, const IntegralPlan& I, double* dev_out, hipStream_t st,
                          const unsigned long long* gate, int want) {
  const int dim = e->p.dimension;
  const int npT = (int)e->pT.size(), nphi = (int)e->phi.size();
  const int ny_out = (dim == 3) ? (int)e->y.size() : 1;
  const int nk = ny_out, nl = (dim == 3) ? 1 : (int)e->eta.size();
  const int nc = e->ncls;
  ReduceArgs ra{};
  ra.slab = e->d_slab; ra.sstride = I.sstride; ra.nsplit = I.fold ? 1 : (int)(I.nsplit + I.nsplit_fb);
  ra.nbx = (int)I.bx; ra.npart = nc; ra.npT = npT; ra.nphi = nphi; ra.nk = nk; ra.nl = nl; ra.ny_out = ny_out; ra.kj = I.P.KJ;
  ra.ntask = I.ntask;
  ra.sorig = e->d_sorig; ra.degen_orig = e->d_degen_orig; ra.prefactor = std::pow(2.0 * M_PI * kHbarC, -3);
  ra.cmem_off = e->d_cmem_off; ra.cmem = e->d_cmem;
  ra.out = dev_out;
  ra.gate = gate; ra.gate_want = want;
  // one wavefront per output when each output sums many (eta node, split) terms and there are few outputs
  if ((long)nl * ra.nsplit >= 128 && I.sstride / nl < (1L << 20)) {
    const long nout = (long)nc * npT * nphi * ny_out;
    hipLaunchKernelGGL(k_reduce_wave, dim3((unsigned)((nout + 3) / 4)), dim3(256), 0, st, ra);
  } else {
    hipLaunchKernelGGL(k_reduce, dim3((unsigned)((I.sstride + 255) / 256)), dim3(256), 0, st, ra);
  }
  HIPCHK(e, hipGetLastError());
  return IS3D_OK;
}

static int launch_end(is3d_engine* e) {
  LaunchCtx& L = e->lc;
  hipStream_t st = L.st;
  double* dev_out = L.dev_out;
  HIPCHK(e, hipSetDevice(e->device));
  if (L.empty) {
    HIPCHK(e, hipEventRecord(e->ev[1], st));
    HIPCHK(e, hipEventRecord(e->ev[2], st));
    HIPCHK(e, hipEventRecord(e->ev[3], st));
    e->launched = true;
    return IS3D_OK;
  }
  const long n = e->ncell;
  const int mode = e->p.df_mode;
  const long wlo = L.wlo, nw = L.nw;
  const PrepArgs& pa = L.pa;
  const dim3 g1((unsigned)std::max(1L, (L.p1 - L.p0 + 255) / 256)), b1(256);
  if (mode == PTMA) {
    hipLaunchKernelGGL(k_famod_b, g1, b1, 0, st, pa, (const double*)e->d_sol);
    HIPCHK(e, hipGetLastError());
  }
  if (mode == PTM) {
    if (!ensure(e->d_renorm, e->renorm_cap, nw * (long)e->nrcls)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(renorm) failed");
    RenormArgs ra{};
    ra.k = pa.k; ra.rec = e->d_rec; ra.aux = e->d_aux; ra.renorm = e->d_renorm;
    ra.mass = e->d_smass; ra.sign = e->d_ssign; ra.degen = e->d_sdegen; ra.baryon = e->d_sbaryon;
    ra.c0 = wlo; ra.n = nw; ra.stride = n;
    ra.npart = e->nrcls; ra.rrep = e->d_rrep;
    const long tot = nw * (long)e->nrcls;
    hipLaunchKernelGGL(k_renorm, dim3((unsigned)std::max(1L, (tot + 255) / 256)), dim3(256), 0, st, ra);
    HIPCHK(e, hipGetLastError());
  }
  HIPCHK(e, hipEventRecord(e->ev[1], st));
  // the integral and the reduction see the window only: records from wlo on, nw cells
  const double* rec_w = e->d_rec + wlo * (long)NREC;
  // --- main integral
  // Grad / RTA-CE F_TS: a surface with cells whose lanes may leave the fast path (k_prep counts them in cnt[4]; none
  // in any tabulated delta-f range) needs the kernels that carry the slow loop, which the F_TS ones do not.  The
  // choice is made on the device: both plans are enqueued, each gated on cnt[4] (gate_closed: the other plan's
  // workgroups return at once, ~10 us), so is3d_launch never waits for the prepass (no host round trip)
  const SpectraPlan P = spectra_plan(e, true);
  e->last_nchunk = 0;
  IntegralPlan I{}, J{};
  int rc = integral_plan(e, P, nw, I);
  if (rc) return rc;
  e->last_nsplit = I.nsplit;
  e->last_nslab = I.slabs();
  const bool gated = mode <= CE && P.ts;
  if (gated) {
    // the fallback plan shares the slab memory: a folded main plan caps its splits at the same footprint
    rc = integral_plan(e, spectra_plan(e, false), nw, J, I.fold ? I.slabs() : 0);
    if (rc) return rc;
  }
  const long slab_need = std::max(I.slabs() * I.sstride, gated ? J.slabs() * J.sstride : 0L);
  if (!ensure(e->d_slab, e->slab_cap, slab_need)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(slabs) failed");
  const unsigned long long* gate = gated ? e->d_cnt + 4 : nullptr;
  rc = enqueue_spectra(e, I, rec_w, nw, st, gate, 0);
  if (!rc && gated) rc = enqueue_spectra(e, J, rec_w, nw, st, gate, 1);
  if (rc) return rc;
  HIPCHK(e, hipEventRecord(e->ev[2], st));
  rc = enqueue_reduce(e, I, dev_out, st, gate, 0);
  if (!rc && gated) rc = enqueue_reduce(e, J, dev_out, st, gate, 1);
  if (rc) return rc;
  HIPCHK(e, hipEventRecord(e->ev[3], st));
  e->launched = true;
  return IS3D_OK;
}

extern "C" int is3d_launch(is3d_engine* e, double* dev_out, void* stream) {
  if (e && e->grp) return is3d::group_launch(e->grp, dev_out, stream);
  if (!e) return IS3D_ERR_ARG;
  if (e->chain_q1 >= 0)
    return e->fail(IS3D_ERR_STATE, "a chain range (is3d_set_chain_range) runs through the staged launch: its first "
                                   "positions need the previous range's boundary states");
  int rc = launch_begin(e, dev_out, stream, 0, -1, 0);
  for (int pass = 0; !rc && e->lc.chained && pass < e->lc.ca.npass; pass++) rc = chain_pass(e, pass);
  if (!rc) rc = chain_end(e);
  return rc ? rc : launch_end(e);
}

// staged launch for the device group (group.h)
int is3d_internal_launch_begin(is3d_engine* e, double* dev_out, void* stream, long q0, long q1, int has_pred) {
  return launch_begin(e, dev_out, stream, q0, q1, has_pred);
}
int is3d_internal_chain_pass(is3d_engine* e, int pass) { return chain_pass(e, pass); }
int is3d_internal_chain_end(is3d_engine* e) { return chain_end(e); }
int is3d_internal_launch_end(is3d_engine* e) { return launch_end(e); }
int is3d_internal_chain_npass(const is3d_engine* e) { return e->lc.chained && !e->lc.empty ? e->lc.ca.npass : 0; }
// boundary slot k (0, 1: pass parity, 2: final) of this engine's chain range: in (from the previous shard) or out
double* is3d_internal_chain_bnd(is3d_engine* e, int out, int slot) {
  if (!e->lc.chained || e->lc.empty) return nullptr;
  const long bw = 4 * e->lc.ca.C + 1;
  return (out ? e->lc.ca.bout : e->lc.ca.bin) + slot * bw;
}
long is3d_internal_chain_bnd_bytes(const is3d_engine* e) { return (4 * e->lc.ca.C + 1) * (long)sizeof(double); }

// ---- staged launch for PTMA warm-start chains split over processes (include/is3d_amd.h) ----------------------------
extern "C" int is3d_set_chain_range(is3d_engine* e, long q0, long q1) {
  if (!e) return IS3D_ERR_ARG;
  if (e->grp) return is3d::group_fail(e->grp, IS3D_ERR_UNSUPPORTED, "a device-list engine splits its chains itself");
  if (q0 < 0 || q1 < 0) { e->chain_q0 = e->chain_q1 = -1; e->win_lo = e->win_hi = -1; return IS3D_OK; }
  if (!e->have_params || e->p.df_mode != PTMA || e->p.famod_chains <= 0)
    return e->fail(IS3D_ERR_STATE, "a chain range needs PTMA (df_mode 5) with famod_chains > 0 set first");
  const long n = e->ncell, C = std::max(1L, std::min<long>(e->p.famod_chains, std::max(n, 1L))), P = (n + C - 1) / C;
  if (q0 > q1 || q1 > P) return e->fail(IS3D_ERR_ARG, "chain range outside the surface's chain positions");
  e->win_lo = std::min(n, q0 * C);
  e->win_hi = std::min(n, q1 * C);
  e->chain_q0 = q0; e->chain_q1 = q1;
  return IS3D_OK;
}

extern "C" int is3d_launch_begin(is3d_engine* e, double* dev_out, void* stream) {
  if (!e) return IS3D_ERR_ARG;
  if (e->grp) return is3d::group_fail(e->grp, IS3D_ERR_UNSUPPORTED, "the staged launch runs on one-device engines");
  if (e->chain_q1 >= 0 && (e->p.df_mode != PTMA || e->p.famod_chains <= 0))
    return e->fail(IS3D_ERR_STATE, "a chain range needs PTMA with famod_chains > 0 (params changed since)");
  const bool range = e->chain_q1 >= 0;
  if (range) {
    // the integration window follows the chain positions under the current famod_chains C (set_params may have
    // changed C since is3d_set_chain_range): cells [q0 C, q1 C), so the ranks' windows still tile the surface
    const long n = e->ncell, C = std::max(1L, std::min<long>(e->p.famod_chains, std::max(n, 1L))), P = (n + C - 1) / C;
    if (e->chain_q1 > P) return e->fail(IS3D_ERR_ARG, "chain range outside the surface's chain positions (famod_chains changed)");
    e->win_lo = std::min(n, e->chain_q0 * C);
    e->win_hi = std::min(n, e->chain_q1 * C);
  }
  return launch_begin(e, dev_out, stream, range ? e->chain_q0 : 0, range ? e->chain_q1 : -1, range && e->chain_q0 > 0);
}
extern "C" int is3d_chain_passes(const is3d_engine* e) { return e && !e->grp ? is3d_internal_chain_npass(e) : 0; }
extern "C" int is3d_chain_pass(is3d_engine* e, int pass) {
  if (!e || e->grp) return IS3D_ERR_ARG;
  if (pass < 0 || pass >= is3d_internal_chain_npass(e)) return e->fail(IS3D_ERR_ARG, "chain pass out of range");
  return chain_pass(e, pass);
}
extern "C" int is3d_chain_end(is3d_engine* e) { return (!e || e->grp) ? IS3D_ERR_ARG : chain_end(e); }
extern "C" int is3d_launch_end(is3d_engine* e) { return (!e || e->grp) ? IS3D_ERR_ARG : launch_end(e); }
extern "C" long is3d_chain_boundary_size(const is3d_engine* e) {
  return (e && !e->grp && e->lc.chained && !e->lc.empty) ? 4 * e->lc.ca.C + 1 : 0;
}
// boundary slot `slot` (0, 1: pass parity, 2: the finisher's) out of this range into dev_buf / from dev_buf into this
// range's incoming slot, on the launch stream (hipMemcpyDefault: a host buffer works too, read after a stream sync)
extern "C" int is3d_chain_boundary_get(is3d_engine* e, int slot, double* dev_buf) {
  if (!e || e->grp || !dev_buf || slot < 0 || slot >= kBndSlots) return e ? e->fail(IS3D_ERR_ARG, "bad chain boundary slot") : IS3D_ERR_ARG;
  const long nb = is3d_chain_boundary_size(e);
  if (nb == 0) return e->fail(IS3D_ERR_STATE, "no chains in the launch in flight");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipMemcpyAsync(dev_buf, is3d_internal_chain_bnd(e, 1, slot), nb * sizeof(double), hipMemcpyDefault, e->lc.st));
  return IS3D_OK;
}
extern "C" int is3d_chain_boundary_put(is3d_engine* e, int slot, const double* dev_buf) {
  if (!e || e->grp || !dev_buf || slot < 0 || slot >= kBndSlots) return e ? e->fail(IS3D_ERR_ARG, "bad chain boundary slot") : IS3D_ERR_ARG;
  const long nb = is3d_chain_boundary_size(e);
  if (nb == 0) return e->fail(IS3D_ERR_STATE, "no chains in the launch in flight");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipMemcpyAsync(is3d_internal_chain_bnd(e, 0, slot), dev_buf, nb * sizeof(double), hipMemcpyDefault, e->lc.st));
  return IS3D_OK;
}

extern "C" int is3d_cell_costs(is3d_engine* e, double* cost) {
  if (e && e->grp) return is3d::group_fail(e->grp, IS3D_ERR_UNSUPPORTED, "is3d_cell_costs: call it on a one-device engine");
  if (!e || !cost) return IS3D_ERR_ARG;
  int rc = finalize_tables(e);
  if (rc) return rc;
  const long n = e->ncell;
  if (n <= 0) return IS3D_OK;
  HIPCHK(e, hipSetDevice(e->device));
  const int mode = e->p.df_mode;
  // private scratch (records, aux, cost, error word, counters), freed on return: a launch in flight keeps its
  // buffers and the error word is3d_finish reports, and a device group's cost prepass over the whole surface
  // (group_set_surface on shard 0) leaves no full-surface-sized buffers behind on that shard
  double* scratch = nullptr;
  const size_t nd = (size_t)(NREC + 9 + 1) * n + 9;
  HIPCHK(e, hipMalloc(&scratch, nd * sizeof(double)));
  double* d_rec = scratch;
  double* d_aux = d_rec + (size_t)NREC * n;
  double* d_cost = d_aux + 9 * (size_t)n;
  int* d_err = (int*)(d_cost + n);
  unsigned long long* d_cnt = (unsigned long long*)(d_cost + n + 1);
  PrepArgs pa{};
  pa.k = make_consts(e); pa.tb = e->dtb; pa.surf = e->d_surf; pa.rec = d_rec; pa.aux = d_aux; pa.n = n;
  pa.c0 = 0; pa.c1 = n;
  pa.err = d_err; pa.cnt = d_cnt;
  const dim3 g1((unsigned)((n + 255) / 256)), b1(256);
  hipError_t er = hipMemsetAsync(d_err, 0, 9 * sizeof(double), nullptr);
  switch (mode) {
    case GRAD: hipLaunchKernelGGL(k_prep<GRAD>, g1, b1, 0, nullptr, pa); break;
    case CE: hipLaunchKernelGGL(k_prep<CE>, g1, b1, 0, nullptr, pa); break;
    case PTM: hipLaunchKernelGGL(k_prep<PTM>, g1, b1, 0, nullptr, pa); break;
    case PTB: hipLaunchKernelGGL(k_prep<PTB>, g1, b1, 0, nullptr, pa); break;
    default: hipLaunchKernelGGL(k_prep<PTMA>, g1, b1, 0, nullptr, pa); break;
  }
  // separable-fallback cells of PTM / PTB relative to a modified cell (config-2 shape, MI355X,
  // tools/fb_cost_probe.py: PTM 1.37-1.43, PTB 1.58-1.80)
  const double fb_cost = mode == PTM ? 1.4 : mode == PTB ? 1.8 : 0.0;
  hipLaunchKernelGGL(k_cell_cost, g1, b1, 0, nullptr, (const double*)d_rec, n, fb_cost, d_cost);
  if (er == hipSuccess) er = hipGetLastError();
  if (er == hipSuccess) er = hipMemcpy(cost, d_cost, n * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipFree(scratch);
  if (er != hipSuccess) return e->fail(IS3D_ERR_DEVICE, std::string("is3d_cell_costs: ") + hipGetErrorString(er));
  return IS3D_OK;
}

extern "C" int is3d_finish(is3d_engine* e) {
  if (e && e->grp) return is3d::group_finish(e->grp);
  if (!e) return IS3D_ERR_ARG;
  if (!e->launched) return e->fail(IS3D_ERR_STATE, "nothing launched");
  HIPCHK(e, hipSetDevice(e->device));
  HIPCHK(e, hipEventSynchronize(e->ev[3]));
  e->launched = false;
  int derr = 0;
  unsigned long long cnt[8];
  HIPCHK(e, hipMemcpy(&derr, e->d_err, sizeof(int), hipMemcpyDeviceToHost));
  HIPCHK(e, hipMemcpy(cnt, e->d_cnt, sizeof(cnt), hipMemcpyDeviceToHost));
  e->st.breakdown = (long)cnt[0]; e->st.pl_negative = (long)cnt[1]; e->st.recon_fail = (long)cnt[2]; e->st.iterations = (long)cnt[3];
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, e->ev[0], e->ev[1]) == hipSuccess) e->st.ms_prepass = ms;
  if (hipEventElapsedTime(&ms, e->ev[1], e->ev[2]) == hipSuccess) e->st.ms_spectra = ms;
  if (hipEventElapsedTime(&ms, e->ev[0], e->ev[3]) == hipSuccess) e->st.ms_total = ms;
  switch (derr) {
    case DF_OK: return IS3D_OK;
    case DF_SPLINE_RANGE: return e->fail(IS3D_ERR_DF_RANGE, "gsl: interp.c: interpolation error (df coefficient spline evaluated outside its table)");
    case DF_TABLE_RANGE: return e->fail(IS3D_ERR_DF_RANGE, "Error: (T,muB) outside df coefficient table. Exiting...");
    case DF_PTB_BARYON: return e->fail(IS3D_ERR_UNSUPPORTED, "Bilinear interpolation error: Jonah df doesn't work for nonzero muB. Exiting..");
    case DF_TS_SLOW: return e->fail(IS3D_ERR_DEVICE, "internal: a scalar-table (F_TS) lane left the fast path (sep_slow_cell bound)");
    default: return e->fail(IS3D_ERR_ARG, "Error: choose df_mode = (1,2,3,4,5)");
  }
}

extern "C" int is3d_calculate_spectra(is3d_engine* e, double* dN_out) {
  if (e && e->grp) return is3d::group_calculate_spectra(e->grp, dN_out);
  if (!e || !dN_out) return e ? e->fail(IS3D_ERR_ARG, "null output") : IS3D_ERR_ARG;
  int rc = finalize_tables(e);
  if (rc) return rc;
  const long outsize = is3d_output_size(e);
  if (!ensure(e->d_out, e->out_cap, outsize)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(output) failed");
  rc = is3d_launch(e, e->d_out, nullptr);
  if (rc) return rc;
  rc = is3d_finish(e);
  if (rc) return rc;
  HIPCHK(e, hipMemcpy(dN_out, e->d_out, outsize * sizeof(double), hipMemcpyDeviceToHost));
  return IS3D_OK;
}

// operation = 0 (SpacetimeDistribution.cpp:31-1250): device prepass + per-(species, cell) yields + binning
// into thread slices; the host then applies the reference's per-species reset (byte-count memset,
// :165-167 / :628-630) and writes the bin-normalised distributions (:407-440).
extern "C" int is3d_calculate_dN_dX(is3d_engine* e, double* dN_taudtaudy, double* dN_2pirdrdy, double* dN_dphidy) {
  if (e && e->grp) return is3d::group_calculate_dN_dX(e->grp, dN_taudtaudy, dN_2pirdrdy, dN_dphidy);
  if (!e) return IS3D_ERR_ARG;
  if (!dN_taudtaudy || !dN_2pirdrdy || !dN_dphidy) return e->fail(IS3D_ERR_ARG, "null output");
  if (!e->have_params) return e->fail(IS3D_ERR_STATE, "is3d_set_params not called");
  if (e->p.df_mode == PTMA) return e->fail(IS3D_ERR_UNSUPPORTED, "calculate_spectra error: no spacetime distribution routine for famod yet");
  if (!e->have_weights) return e->fail(IS3D_ERR_STATE, "is3d_set_momentum_weights not called");
  if (!e->have_bins) return e->fail(IS3D_ERR_STATE, "is3d_set_spacetime_bins not called");
  int rc = finalize_tables(e);
  if (rc) return rc;
  HIPCHK(e, hipSetDevice(e->device));
  hipStream_t st = nullptr;
  const long n = e->ncell;
  const int mode = e->p.df_mode, dim = e->p.dimension;
  const int np = (int)e->mass.size(), npT = (int)e->pT.size(), nphi = (int)e->phi.size();
  const int nk = (dim == 3) ? (int)e->y.size() : 1, nl = (dim == 3) ? 1 : (int)e->eta.size();
  const is3d_spacetime_bins& B = e->bins;
  const long C = std::max(1, B.threads);
  const int carry = B.threads >= 1;
  const long nb[3] = {B.tau_bins, B.r_bins, B.phip_bins};
  const long nent = C * (nb[0] + nb[1] + nb[2]);
  e->st = is3d_stats{};
  e->st.cells = n;
  std::vector<double> part((size_t)np * nent, 0.0);
  HIPCHK(e, hipMemsetAsync(e->d_err, 0, sizeof(int), st));
  HIPCHK(e, hipMemsetAsync(e->d_cnt, 0, 8 * sizeof(unsigned long long), st));
  HIPCHK(e, hipEventRecord(e->ev[0], st));
  if (n > 0) {
    if (!ensure(e->d_rec, e->rec_cap, (long)NREC * n)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(records) failed");
    if (!ensure(e->d_aux, e->aux_cap, 9L * n)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(aux) failed");
    PrepArgs pa{};
    pa.k = make_consts(e); pa.k.operation = 0;
    pa.tb = e->dtb; pa.surf = e->d_surf; pa.rec = e->d_rec; pa.aux = e->d_aux; pa.n = n;
    pa.c0 = 0; pa.c1 = n;
    pa.err = e->d_err; pa.cnt = e->d_cnt;
    const dim3 g1((unsigned)((n + 255) / 256)), b1(256);
    switch (mode) {
      case GRAD: hipLaunchKernelGGL(k_prep<GRAD>, g1, b1, 0, st, pa); break;
      case CE: hipLaunchKernelGGL(k_prep<CE>, g1, b1, 0, st, pa); break;
      case PTM: hipLaunchKernelGGL(k_prep<PTM>, g1, b1, 0, st, pa); break;
      default: hipLaunchKernelGGL(k_prep<PTB>, g1, b1, 0, st, pa); break;
    }
    HIPCHK(e, hipGetLastError());
    if (mode == PTM) {
      if (!ensure(e->d_renorm, e->renorm_cap, n * (long)e->nrcls)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(renorm) failed");
      RenormArgs ra{};
      ra.k = pa.k; ra.rec = e->d_rec; ra.aux = e->d_aux; ra.renorm = e->d_renorm;
      ra.mass = e->d_smass; ra.sign = e->d_ssign; ra.degen = e->d_sdegen; ra.baryon = e->d_sbaryon;
      ra.c0 = 0; ra.n = n; ra.stride = n;
      ra.npart = e->nrcls; ra.rrep = e->d_rrep;
      const long tot = n * (long)e->nrcls;
      hipLaunchKernelGGL(k_renorm, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, ra);
      HIPCHK(e, hipGetLastError());
    }
  }
  HIPCHK(e, hipEventRecord(e->ev[1], st));
  if (n > 0) {
    // --- per-(species, cell) yields
    const int KJ = spectra_kj(nphi);
    const int njb = (nphi + KJ - 1) / KJ;
    DndxArgs da{};
    const int nc = e->ncls;    // lane species: the integrand classes (k_stbin scales and writes the members)
    da.ntask = nk * njb * nl;
    da.Sl = std::min(nc, 64);
    da.Yl = 64 / da.Sl;
    da.nbx = (nc + da.Sl - 1) / da.Sl;
    static_assert(is3d::kern::kTile % IS3D_DNDX_TILE_MOD == 0 && is3d::kern::kTile % IS3D_DNDX_TILE == 0,
                  "k_dndx's cells per workgroup (multiples of kTile) hold whole record tiles");
    long cpw = 4L * kTile;
    if ((long)da.nbx * ((n + cpw - 1) / cpw) < 4096) cpw = kTile;
    da.cells_per_wg = cpw;
    da.nchunk = (n + cpw - 1) / cpw;
    if (!ensure(e->d_ycell, e->ycell_cap, (long)nc * n)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(cell yields) failed");
    da.rec = e->d_rec; da.n = n; da.renorm = e->d_renorm; da.rcls = e->d_crcls; da.nrcls = e->nrcls; da.ycell = e->d_ycell;
    da.smass = e->d_cmass; da.ssign = e->d_csign; da.sbaryon = e->d_cbaryon;
    da.pT = e->d_pT; da.pTw = e->d_pTw; da.cphi = e->d_cphi; da.sphi = e->d_sphi; da.phiw = e->d_phiw;
    da.yv = e->d_y; da.etav = e->d_eta; da.etaw = e->d_etaw;
    da.npart = nc; da.npT = npT; da.nphi = nphi; da.nk = nk; da.nl = nl; da.nq = nk * nl; da.njb = njb; da.dim = dim;
    const size_t nphp = (size_t)njb * KJ;
    // kernels.h k_dndx's layout: records, trig / {pc, ps} / phi weights, {b', Phi} rows (not in the modified launch:
    // IS3D_MOD_TABLES), Qv rows, per-lane cell sums, grid, y-term rows, exp table, PTM's renorm factors [kTile][Sl]
    auto dndx_lds = [&](bool modmain, bool fb = false) {
      const bool bp = !(modmain && IS3D_MOD_TABLES);
      // kernels.h dndx_tile: the launch's record tile
      const size_t kTile = fb ? is3d::kern::kTile : modmain ? IS3D_DNDX_TILE_MOD : IS3D_DNDX_TILE;
      return sizeof(double) * ((size_t)kTile * NREC + 2 * nphp + 2 * nphp + nphp + (bp ? 2 : 0) * (size_t)kTile * nphp +
                               (modmain && IS3D_DNDX_PDM && KJ % 4 == 0 ? 2 : 1) * (size_t)kTile * nphp +
                               (size_t)kTile * kBlock + (size_t)(nk + 2 * nl) +
                               (size_t)kTile * da.nq * kYRowLY + (size_t)(modmain ? is3d::kModTabN : kExpTabN) +
                               (mode == PTM ? (size_t)kTile * da.Sl : 0));
    };
    const size_t shmem = dndx_lds(mode >= PTM), shmem_fb = dndx_lds(false, true);
    if (std::max(shmem, shmem_fb) > 160 * 1024) return e->fail(IS3D_ERR_ARG, "momentum grid too large for the LDS tile");
    const long nwg = (long)da.nbx * da.nchunk;
    if (nwg > 0x7fffffffL) return e->fail(IS3D_ERR_ARG, "surface too large for one dN/dX launch");
    const int kflags = (e->p.regulate_deltaf ? F_REG : 0) | (e->p.outflow ? F_OUT : 0);
    switch (mode) {
      case GRAD: launch_dndx<GRAD>(dim3((unsigned)nwg), shmem, st, da, kflags, KJ); break;
      case CE: launch_dndx<CE>(dim3((unsigned)nwg), shmem, st, da, kflags, KJ); break;
      case PTM: launch_dndx<PTM>(dim3((unsigned)nwg), shmem, st, da, kflags, KJ); break;
      default: launch_dndx<PTB>(dim3((unsigned)nwg), shmem, st, da, kflags, KJ); break;
    }
    HIPCHK(e, hipGetLastError());
    if (mode >= PTM) {
      // the separable-fallback lanes of the cells k_fbwrite lists (breakdown, narrow rapidity windows) in their own
      // launch (kernels.h k_dndx F_FB), added to ycell; the list's length stays on the device, so the grid is sized
      // for the whole surface and the workgroups split whatever the list holds
      if (!ensure(e->d_fb, e->fb_cap, n + 1 + kFbBlocks)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(fallback list) failed");
      enqueue_fbscan((const double*)e->d_rec, n, e->d_fb, st);
      DndxArgs fa = da;
      fa.fbcells = e->d_fb + 1; fa.fbcount = e->d_fb;
      fa.nchunk = std::max(1L, std::min(da.nchunk, (4096L + da.nbx - 1) / da.nbx));
      const long nfw = (long)da.nbx * fa.nchunk;
      if (mode == PTM) launch_dndx<PTM>(dim3((unsigned)nfw), shmem_fb, st, fa, kflags | F_FB, KJ);
      else launch_dndx<PTB>(dim3((unsigned)nfw), shmem_fb, st, fa, kflags | F_FB, KJ);
      HIPCHK(e, hipGetLastError());
    }
    e->ycell_n = n;
  } else {
    e->ycell_n = 0;
  }
  HIPCHK(e, hipEventRecord(e->ev[2], st));
  if (n > 0) {
    // --- bin keys on the device, CSR (thread slice, bin) -> cells on the host, sums on the device
    if (!ensure(e->d_keys, e->keys_cap, 3 * n)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(keys) failed");
    KeyArgs ka{};
    ka.tau = e->d_surf; ka.x = e->d_surf + n; ka.y = e->d_surf + 2 * n; ka.n = n;
    ka.tau_min = B.tau_min; ka.tau_width = (B.tau_max - B.tau_min) / (double)B.tau_bins;
    ka.r_min = B.r_min; ka.r_width = (B.r_max - B.r_min) / (double)B.r_bins;
    ka.phip_width = 2.0 * M_PI / (double)B.phip_bins;
    ka.tau_bins = B.tau_bins; ka.r_bins = B.r_bins; ka.phip_bins = B.phip_bins; ka.keys = e->d_keys;
    hipLaunchKernelGGL(k_stkeys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ka);
    HIPCHK(e, hipGetLastError());
    std::vector<int> keys((size_t)3 * n);
    HIPCHK(e, hipMemcpy(keys.data(), e->d_keys, keys.size() * sizeof(int), hipMemcpyDeviceToHost));
    std::vector<long> offs((size_t)nent + 1, 0);
    long off_d[3] = {0, C * nb[0], C * (nb[0] + nb[1])};
    for (int d = 0; d < 3; d++)
      for (long c = 0; c < n; c++) {
        const int kb = keys[(size_t)d * n + c];
        if (kb >= 0) offs[off_d[d] + (c % C) * nb[d] + kb + 1]++;
      }
    for (long i = 0; i < nent; i++) offs[i + 1] += offs[i];
    std::vector<int> perm((size_t)std::max(offs[nent], 1L));
    std::vector<long> fill(offs.begin(), offs.end() - 1);
    for (int d = 0; d < 3; d++)
      for (long c = 0; c < n; c++) {
        const int kb = keys[(size_t)d * n + c];
        if (kb >= 0) perm[fill[off_d[d] + (c % C) * nb[d] + kb]++] = (int)c;
      }
    if (!ensure(e->d_perm, e->perm_cap, (long)perm.size())) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(perm) failed");
    if (!ensure(e->d_offs, e->offs_cap, nent + 1)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(offsets) failed");
    if (!ensure(e->d_part, e->part_cap, (long)np * nent)) return e->fail(IS3D_ERR_DEVICE, "hipMalloc(bins) failed");
    HIPCHK(e, hipMemcpy(e->d_perm, perm.data(), perm.size() * sizeof(int), hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_offs, offs.data(), offs.size() * sizeof(long), hipMemcpyHostToDevice));
    BinArgs ba{};
    ba.ycell = e->d_ycell; ba.n = n; ba.npart = np;
    ba.perm = e->d_perm; ba.offs = e->d_offs; ba.nent = nent;
    ba.sorig = e->d_sorig; ba.sdegen = e->d_sdegen; ba.prefactor = std::pow(2.0 * M_PI * kHbarC, -3);
    ba.scls = e->d_scls;
    ba.part = e->d_part;
    const long nthr = nent * np;
    hipLaunchKernelGGL(k_stbin, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, st, ba);
    HIPCHK(e, hipGetLastError());
  }
  HIPCHK(e, hipEventRecord(e->ev[3], st));
  HIPCHK(e, hipEventSynchronize(e->ev[3]));
  int derr = 0;
  HIPCHK(e, hipMemcpy(&derr, e->d_err, sizeof(int), hipMemcpyDeviceToHost));
  if (n > 0) HIPCHK(e, hipMemcpy(part.data(), e->d_part, part.size() * sizeof(double), hipMemcpyDeviceToHost));
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, e->ev[0], e->ev[1]) == hipSuccess) e->st.ms_prepass = ms;
  if (hipEventElapsedTime(&ms, e->ev[1], e->ev[2]) == hipSuccess) e->st.ms_spectra = ms;
  if (hipEventElapsedTime(&ms, e->ev[0], e->ev[3]) == hipSuccess) e->st.ms_total = ms;
  switch (derr) {
    case DF_OK: break;
    case DF_SPLINE_RANGE: return e->fail(IS3D_ERR_DF_RANGE, "gsl: interp.c: interpolation error (df coefficient spline evaluated outside its table)");
    case DF_TABLE_RANGE: return e->fail(IS3D_ERR_DF_RANGE, "Error: (T,muB) outside df coefficient table. Exiting...");
    case DF_PTB_BARYON: return e->fail(IS3D_ERR_UNSUPPORTED, "Bilinear interpolation error: Jonah df doesn't work for nonzero muB. Exiting..");
    default: return e->fail(IS3D_ERR_ARG, "Error: set df_mode = (1,2) in parameters.dat");
  }
  // --- the reference's per-species thread-slice reset and bin normalisation
  const double two_pi = 2.0 * M_PI;
  const double width[3] = {(B.tau_max - B.tau_min) / (double)B.tau_bins, (B.r_max - B.r_min) / (double)B.r_bins,
                           two_pi / (double)B.phip_bins};
  double* outs[3] = {dN_taudtaudy, dN_2pirdrdy, dN_dphidy};
  long off = 0;
  for (int d = 0; d < 3; d++) {
    const long bins = nb[d];
    std::vector<double> all((size_t)C * bins, 0.0);
    for (int k = 0; k < np; k++) {
      if (carry) std::memset(all.data(), 0, (size_t)(C * bins));   // bytes, not doubles (:165-167)
      else std::fill(all.begin(), all.end(), 0.0);
      const double* pk = part.data() + (size_t)k * nent + off;
      for (long t = 0; t < C; t++)
        for (long i = 0; i < bins; i++) all[i + t * bins] += pk[t * bins + i];
      for (long i = 0; i < bins; i++) {
        double acc = 0.0;
        for (long t = 0; t < C; t++) acc += all[i + t * bins];
        double norm = width[d];
        if (d == 0) norm = (B.tau_min + width[0] * ((double)i + 0.5)) * width[0];
        else if (d == 1) norm = two_pi * (B.r_min + width[1] * ((double)i + 0.5)) * width[1];
        outs[d][(size_t)k * bins + i] = acc / norm;
      }
    }
    off += C * bins;
  }
  return IS3D_OK;
}

extern "C" int is3d_get_cell_yields(const is3d_engine* e, double* dN_dy_cell) {
  if (e && e->grp) return is3d::group_get_cell_yields(e->grp, dN_dy_cell);
  if (!e || !dN_dy_cell) return IS3D_ERR_ARG;
  if (e->ycell_n < 0) return IS3D_ERR_STATE;
  const long n = e->ycell_n;
  const int np = (int)e->mass.size();
  if (n == 0) return IS3D_OK;
  std::vector<double> y((size_t)e->ncls * n);
  if (hipSetDevice(e->device) != hipSuccess) return IS3D_ERR_DEVICE;
  if (hipMemcpy(y.data(), e->d_ycell, y.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return IS3D_ERR_DEVICE;
  const double pref = std::pow(2.0 * M_PI * kHbarC, -3);
  for (int s = 0; s < np; s++) {
    const int so = e->order[s];
    for (long c = 0; c < n; c++) dN_dy_cell[(size_t)so * n + c] = pref * e->degen[so] * y[(size_t)e->scls[s] * n + c];
  }
  return IS3D_OK;
}

extern "C" int is3d_get_stats(const is3d_engine* e, is3d_stats* out) {
  if (e && e->grp) return out ? is3d::group_get_stats(e->grp, out) : IS3D_ERR_ARG;
  if (!e || !out) return IS3D_ERR_ARG;
  *out = e->st;
  return IS3D_OK;
}

extern "C" int is3d_evaluate_df_coefficients(is3d_engine* e, double T, double muB, double E, double P, double bulkPi,
                                             double* out15) {
  if (e && e->grp) return out15 ? is3d::group_evaluate_df_coefficients(e->grp, T, muB, E, P, bulkPi, out15) : IS3D_ERR_ARG;
  if (!e || !out15) return IS3D_ERR_ARG;
  int rc = finalize_tables(e);
  if (rc) return rc;
  HIPCHK(e, hipSetDevice(e->device));
  double* d = dalloc<double>(16);
  if (!d) return e->fail(IS3D_ERR_DEVICE, "hipMalloc failed");
  hipLaunchKernelGGL(k_df_eval, dim3(1), dim3(1), 0, 0, e->dtb, T, muB, E, P, bulkPi, d, (int*)(d + 15));
  hipError_t h = hipDeviceSynchronize();
  int derr = 0;
  if (h == hipSuccess) h = hipMemcpy(out15, d, 15 * sizeof(double), hipMemcpyDeviceToHost);
  if (h == hipSuccess) h = hipMemcpy(&derr, d + 15, sizeof(int), hipMemcpyDeviceToHost);
  dfree(d);
  if (h != hipSuccess) return hip_fail(e, h, "df eval");
  if (derr == DF_SPLINE_RANGE || derr == DF_TABLE_RANGE) return e->fail(IS3D_ERR_DF_RANGE, "df coefficient evaluated out of range");
  if (derr) return e->fail(IS3D_ERR_ARG, "df coefficient error");
  return IS3D_OK;
}

extern "C" int is3d_total_yield(is3d_engine* e, const double* plasma, double y_cut, double* n_total,
                                double* densities) {
  if (e && e->grp) return is3d::group_total_yield(e->grp, plasma, y_cut, n_total, densities);
  if (!e || !plasma || !n_total) return IS3D_ERR_ARG;
  int rc = finalize_tables(e);
  if (rc) return rc;
  if (!e->have_gla || e->gla_alpha < 4) return e->fail(IS3D_ERR_STATE, "is3d_set_gauss_laguerre: alpha = 1..3 tables needed");
  if (e->gla_pts > 64) return e->fail(IS3D_ERR_ARG, "Gauss-Laguerre table longer than 64 points");
  HIPCHK(e, hipSetDevice(e->device));
  const int np = (int)e->mass.size();
  const long n = e->ncell;
  const long nb = (n + 255) / 256;
  double* d = dalloc<double>(3 * (size_t)np + (size_t)std::max(nb, 1L) + 1);
  if (!d) return e->fail(IS3D_ERR_DEVICE, "hipMalloc failed");
  HIPCHK(e, hipMemset(e->d_err, 0, sizeof(int)));
  DensArgs da{};
  da.tb = e->dtb; da.gla = e->d_gla; da.gla_alpha = e->gla_alpha; da.gla_pts = e->gla_pts;
  da.T = plasma[0]; da.E = plasma[1]; da.P = plasma[2]; da.muB = plasma[3]; da.nB = plasma[4];
  da.smass = e->d_smass; da.ssign = e->d_ssign; da.sdegen = e->d_sdegen; da.sbaryon = e->d_sbaryon; da.sorig = e->d_sorig;
  da.npart = np; da.df_mode = e->p.df_mode; da.two_pi2_hbarC3 = 2.0 * std::pow(M_PI, 2) * std::pow(kHbarC, 3);
  da.dens = d; da.err = e->d_err;
  hipLaunchKernelGGL(k_densities, dim3((unsigned)np), dim3(64), 0, 0, da);
  hipError_t h = hipGetLastError();
  std::vector<double> part((size_t)std::max(nb, 1L), 0.0);
  if (h == hipSuccess && n > 0) {
    YieldArgs ya{};
    ya.k = make_consts(e); ya.tb = e->dtb; ya.surf = e->d_surf; ya.n = n; ya.dens = d; ya.npart = np;
    ya.partial = d + 3 * (size_t)np; ya.err = e->d_err;
    hipLaunchKernelGGL(k_yield, dim3((unsigned)nb), dim3(256), 0, 0, ya);
    h = hipGetLastError();
  }
  if (h == hipSuccess) h = hipDeviceSynchronize();
  int derr = 0;
  if (h == hipSuccess) h = hipMemcpy(&derr, e->d_err, sizeof(int), hipMemcpyDeviceToHost);
  if (h == hipSuccess && n > 0) h = hipMemcpy(part.data(), d + 3 * (size_t)np, nb * sizeof(double), hipMemcpyDeviceToHost);
  if (h == hipSuccess && densities) h = hipMemcpy(densities, d, 3 * (size_t)np * sizeof(double), hipMemcpyDeviceToHost);
  dfree(d);
  if (h != hipSuccess) return hip_fail(e, h, "total yield");
  if (derr == DF_SPLINE_RANGE) return e->fail(IS3D_ERR_DF_RANGE, "gsl: interpolation error (df coefficient spline evaluated out of range)");
  if (derr == DF_TABLE_RANGE) return e->fail(IS3D_ERR_DF_RANGE, "Error: (T,muB) outside df coefficient table");
  if (derr == DF_PTB_BARYON) return e->fail(IS3D_ERR_UNSUPPORTED, "Bilinear interpolation error: Jonah df doesn't work for nonzero muB. Exiting..");
  if (derr) return e->fail(IS3D_ERR_ARG, "df coefficient error");
  double Ntot = 0.0;
  for (long b = 0; b < nb; b++) Ntot += part[b];
  if (e->p.dimension == 2) Ntot *= 2.0 * y_cut;     // :628-631
  *n_total = Ntot;
  return IS3D_OK;
}

extern "C" int is3d_get_jonah_table(const is3d_engine* e, double* l2, double* z, double* bp, double* bpmax) {
  if (e && e->grp) return is3d::group_get_jonah_table(e->grp, l2, z, bp, bpmax);
  if (!e || e->jx.size() != 301) return IS3D_ERR_STATE;
  std::copy(e->jl2.begin(), e->jl2.end(), l2);
  std::copy(e->jz.begin(), e->jz.end(), z);
  std::copy(e->jx.begin(), e->jx.end(), bp);
  *bpmax = e->bp_max;
  return IS3D_OK;
}

extern "C" int is3d_surface_averages(long n, const is3d_surface* s, int include_baryon, double* out) {
  if (!s || !out || n <= 0) return IS3D_ERR_ARG;
  double T_avg = 0, E_avg = 0, P_avg = 0, muB_avg = 0, nB_avg = 0, vol = 0;
  for (long i = 0; i < n; i++) {
    const double tau = s->tau[i], tau2 = tau * tau, ux = s->ux[i], uy = s->uy[i], un = s->un[i];
    const double ut = std::sqrt(1. + ux * ux + uy * uy + tau2 * un * un);
    const double dat = s->dat[i], dax = s->dax[i], day = s->day[i], dan = s->dan[i];
    const double uds = ut * dat + ux * dax + uy * day + un * dan;
    const double ds_ds = dat * dat - dax * dax - day * day - dan * dan / tau2;
    const double ds_max = std::fabs(uds) + std::sqrt(std::fabs(uds * uds - ds_ds));
    const double muB = (include_baryon && s->muB) ? s->muB[i] : 0.0;
    const double nB = (include_baryon && s->nB) ? s->nB[i] : 0.0;
    vol += ds_max;
    E_avg += (s->E[i] * ds_max); T_avg += (s->T[i] * ds_max); P_avg += (s->P[i] * ds_max);
    muB_avg += (muB * ds_max); nB_avg += (nB * ds_max);
  }
  const double v[5] = {T_avg / vol, E_avg / vol, P_avg / vol, muB_avg / vol, nB_avg / vol};
  for (int k = 0; k < 5; k++) {   // ofstream << setprecision(15) then fscanf %lf (readindata.cpp:364-366, :104-119)
    char buf[64];
    std::snprintf(buf, sizeof(buf), "%.15g", v[k]);
    out[k] = std::strtod(buf, nullptr);
  }
  return IS3D_OK;
}

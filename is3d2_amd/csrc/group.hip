// group.hip -- the multi-device engine behind is3d_create_devices (see group.h).
//
// Partitioning: contiguous cell windows, one per device, balanced by an estimated cost --
// a cell with u.dsigma <= 0 is skipped by every kernel (MomentumSpectra.cpp:132; it costs only its record
// prep), any other cell costs one unit.  PTMA with the reference's warm-start chains (famod_chains = C > 0,
// MomentumSpectra.cpp:1308-1364) is a serial recurrence over the whole surface (chain c = cells c, c + C, ...):
// every device holds the whole surface, its window is a range of chain positions [q0, q1) (cells [q0 C, q1 C)),
// and it solves only those positions' Newton steps -- the segmented solve of engine.hip k_chain_pass, with the
// first segment of each chain starting from the end state the previous device pushes after every pass (a peer
// copy of 4 C + 1 doubles) and a sequential finisher hand-off -- so the solutions are the single-device ones
// bit for bit while each device does 1/K of the prepass (IS3D_CHAIN_DIST=0: every device walks every chain).
// Reduction: one ncclAllReduce of the N_s x N_pT x N_phi x N_y float64 spectra over the device outputs on
// the shard streams (RCCL over xGMI), or peer copy + fixed-order add on the first device when the list
// repeats a GPU.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "group.h"

namespace is3d {

namespace {
__global__ __launch_bounds__(256) void k_accum(double* __restrict__ out, const double* __restrict__ add, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) out[i] += add[i];
}
}  // namespace

struct Group {
  std::vector<is3d_engine*> sh;       // shard engines, one per listed device
  std::vector<int> dev;
  std::vector<hipStream_t> st;        // shard k > 0 launches on st[k]; shard 0 on the caller's stream
  std::vector<hipEvent_t> done;       // shard k's work (incl. its reduction step) enqueued up to here
  std::vector<ncclComm_t> comm;       // one communicator per device when every device is distinct
  bool nccl = false;
  std::vector<long> lo, hi;           // cell window of each shard
  bool full = false;                  // every shard holds the whole surface (PTMA warm-start chains)
  std::vector<long> q0, q1;           // full: chain positions of each shard's window (cells [q0 C, q1 C))
  std::vector<hipEvent_t> evE, evF;   // distributed chains: boundary pushed (E) / pass done (F), per shard
  bool dist_chain = false;            // the launch in flight split the chains over the shards
  long ncell = 0;
  is3d_params p{};
  bool have_params = false;
  int np = 0;                         // chosen species
  is3d_spacetime_bins bins{};
  bool have_bins = false;
  std::vector<double*> buf;           // per-shard output buffers (shard 0: the caller's dev_out)
  double* scratch = nullptr;          // device-0 staging buffer of the copy reduction
  long buf_n = 0;
  double* d_out = nullptr; long out_n = 0;   // group_calculate_spectra's device-0 output
  hipStream_t cur0 = nullptr;         // shard 0's stream of the launch in flight
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool launched = false;
  is3d_stats stats{};
  std::string err;
  int fail(int code, const std::string& m) { err = m; return code; }
  int shard_fail(int k, int rc) {
    err = "device " + std::to_string(dev[k]) + ": " + is3d_last_error(sh[k]);
    return rc;
  }
};

static bool needs_full(const Group* g) { return g->have_params && g->p.df_mode == 5 && g->p.famod_chains > 0; }
// the surface was split for other params (PTMA warm-start chains on / off since is3d_set_surface): the windows
// and what each shard holds no longer match what the params need
static bool stale_split(const Group* g) { return g->sh.size() > 1 && g->ncell > 0 && g->full != needs_full(g); }
static const char* kStaleSplit = "the params changed whether every device needs the whole surface (PTMA warm-start "
                                 "chains): set the surface again";

Group* group_create(int n, const int* devices, std::string& err) {
  if (n <= 0 || !devices) { err = "empty device list"; return nullptr; }
  Group* g = new Group();
  g->dev.assign(devices, devices + n);
  for (int k = 0; k < n; k++) {
    is3d_engine* e = is3d_create(devices[k]);
    if (!e) {
      err = "is3d_create(" + std::to_string(devices[k]) + ") failed";
      group_destroy(g);
      return nullptr;
    }
    g->sh.push_back(e);
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;
    if (hipSetDevice(devices[k]) != hipSuccess || (k > 0 && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) ||
        hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      err = "stream / event creation failed on device " + std::to_string(devices[k]);
      group_destroy(g);
      return nullptr;
    }
    g->st.push_back(s);
    g->done.push_back(ev);
    hipEvent_t e1 = nullptr, e2 = nullptr;
    if (hipEventCreateWithFlags(&e1, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e2, hipEventDisableTiming) != hipSuccess) {
      err = "event creation failed on device " + std::to_string(devices[k]);
      group_destroy(g);
      return nullptr;
    }
    g->evE.push_back(e1);
    g->evF.push_back(e2);
  }
  (void)hipSetDevice(devices[0]);
  (void)hipEventCreate(&g->ev0);
  (void)hipEventCreate(&g->ev1);
  // RCCL needs distinct devices (one rank per GPU); IS3D_REDUCE=copy forces the copy reduction, and
  // IS3D_REDUCE=rccl also takes RCCL for a single device (a one-rank communicator: exercises the path)
  const char* mode = std::getenv("IS3D_REDUCE");
  bool distinct = true;
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++) distinct = distinct && devices[a] != devices[b];
  const bool want = (mode && !std::strcmp(mode, "rccl")) || ((!mode || std::strcmp(mode, "copy")) && n > 1);
  if (want && distinct) {
    g->comm.assign(n, nullptr);
    g->nccl = ncclCommInitAll(g->comm.data(), n, devices) == ncclSuccess;
    if (!g->nccl) g->comm.clear();
  }
  return g;
}

void group_destroy(Group* g) {
  if (!g) return;
  for (size_t k = 0; k < g->sh.size(); k++) {
    (void)hipSetDevice(g->dev[k]);
    (void)hipDeviceSynchronize();
    if (k > 0 && k < g->buf.size() && g->buf[k]) (void)hipFree(g->buf[k]);
  }
  for (auto c : g->comm) if (c) ncclCommDestroy(c);
  for (size_t k = 0; k < g->st.size(); k++) {
    (void)hipSetDevice(g->dev[k]);
    if (g->st[k]) (void)hipStreamDestroy(g->st[k]);
    if (g->done[k]) (void)hipEventDestroy(g->done[k]);
    if (k < g->evE.size() && g->evE[k]) (void)hipEventDestroy(g->evE[k]);
    if (k < g->evF.size() && g->evF[k]) (void)hipEventDestroy(g->evF[k]);
  }
  if (!g->dev.empty()) {
    (void)hipSetDevice(g->dev[0]);
    if (g->scratch) (void)hipFree(g->scratch);
    if (g->d_out) (void)hipFree(g->d_out);
    if (g->ev0) (void)hipEventDestroy(g->ev0);
    if (g->ev1) (void)hipEventDestroy(g->ev1);
  }
  for (auto* e : g->sh) is3d_destroy(e);
  delete g;
}

const char* group_error(const Group* g) { return g ? g->err.c_str() : "null group"; }

// the same call on every shard, in order; the first failure is the group's
template <class F>
static int each(Group* g, F f) {
  for (size_t k = 0; k < g->sh.size(); k++) {
    const int rc = f(g->sh[k]);
    if (rc) return g->shard_fail((int)k, rc);
  }
  return IS3D_OK;
}

// the same call on every shard from one host thread per shard (synchronous per-shard work: uploads,
// operation 0 / 2 passes), first failure in shard order
template <class F>
static int each_parallel(Group* g, F f) {
  const int n = (int)g->sh.size();
  std::vector<int> rc(n, IS3D_OK);
  std::vector<std::thread> th;
  for (int k = 0; k < n; k++) th.emplace_back([&, k] { rc[k] = f(k); });
  for (auto& t : th) t.join();
  for (int k = 0; k < n; k++) if (rc[k]) return g->shard_fail(k, rc[k]);
  return IS3D_OK;
}

int group_set_params(Group* g, const is3d_params* p) {
  const int rc = each(g, [&](is3d_engine* e) { return is3d_set_params(e, p); });
  if (!rc) { g->p = *p; g->have_params = true; }
  return rc;
}
int group_set_tuning(Group* g, const char* key, long value) {
  return each(g, [&](is3d_engine* e) { return is3d_set_tuning(e, key, value); });
}
long group_get_tuning(const Group* g, const char* key) {
  if (std::strcmp(key, "phitab_chunks")) return is3d_get_tuning(g->sh[0], key);
  long m = 0;
  for (auto* e : g->sh) m = std::max(m, is3d_get_tuning(e, key));
  return m;
}
int group_set_species(Group* g, int n, const double* m, const double* s, const double* d, const double* b) {
  const int rc = each(g, [&](is3d_engine* e) { return is3d_set_species(e, n, m, s, d, b); });
  if (!rc) g->np = n;
  return rc;
}
int group_set_species_classes(Group* g, int on) {
  return each(g, [&](is3d_engine* e) { return is3d_set_species_classes(e, on); });
}
int group_species_integrated(Group* g) {
  const int n = is3d_species_integrated(g->sh[0]);
  return n < 0 ? -g->shard_fail(0, -n) : n;
}
int group_fail(Group* g, int code, const char* msg) { return g->fail(code, msg); }
int group_set_pdg(Group* g, int n, const double* m, const double* s, const double* d, const double* b) {
  return each(g, [&](is3d_engine* e) { return is3d_set_pdg(e, n, m, s, d, b); });
}
int group_set_momentum_grid(Group* g, int npT, const double* pT, int nphi, const double* phi, int ny, const double* y,
                            int neta, const double* eta, const double* eta_w) {
  return each(g, [&](is3d_engine* e) { return is3d_set_momentum_grid(e, npT, pT, nphi, phi, ny, y, neta, eta, eta_w); });
}
int group_set_momentum_weights(Group* g, const double* a, const double* b) {
  return each(g, [&](is3d_engine* e) { return is3d_set_momentum_weights(e, a, b); });
}
int group_set_spacetime_bins(Group* g, const is3d_spacetime_bins* b) {
  const int rc = each(g, [&](is3d_engine* e) { return is3d_set_spacetime_bins(e, b); });
  if (!rc) { g->bins = *b; g->have_bins = true; }
  return rc;
}
int group_set_gauss_laguerre(Group* g, int alpha, int points, const double* r, const double* w) {
  return each(g, [&](is3d_engine* e) { return is3d_set_gauss_laguerre(e, alpha, points, r, w); });
}
int group_set_df_tables(Group* g, int nT, int nmuB, const double* T, const double* muB, const double* tab, double T_avg) {
  return each(g, [&](is3d_engine* e) { return is3d_set_df_tables(e, nT, nmuB, T, muB, tab, T_avg); });
}

// contiguous windows of ~equal estimated cost: u.dsigma <= 0 cells cost kSkipCost, the rest 1 -- or, when
// `cost` is given (is3d_cell_costs on the whole surface: PTM / PTB separable-fallback cells), those costs
static void balance(Group* g, long n, const double* tau, const double* dat, const double* dax, const double* day,
                    const double* dan, const double* ux, const double* uy, const double* un,
                    const double* cost = nullptr) {
  const int K = (int)g->sh.size();
  std::vector<double> pre((size_t)n + 1, 0.0);
  for (long c = 0; c < n; c++) {
    if (cost) { pre[c + 1] = pre[c] + cost[c]; continue; }
    const double t2 = tau[c] * tau[c];
    const double ut = std::sqrt(1.0 + ux[c] * ux[c] + uy[c] * uy[c] + t2 * un[c] * un[c]);
    const bool live = ut * dat[c] + ux[c] * dax[c] + uy[c] * day[c] + un[c] * dan[c] > 0.0;
    pre[c + 1] = pre[c] + (live ? 1.0 : kSkipCost);
  }
  g->lo.assign(K, 0);
  g->hi.assign(K, n);
  long c = 0;
  for (int k = 0; k < K; k++) {
    g->lo[k] = c;
    if (k == K - 1) { c = n; }
    else {
      const double target = pre[n] * (double)(k + 1) / K;
      c = std::lower_bound(pre.begin() + c, pre.end(), target) - pre.begin();
      c = std::min(std::max(c, g->lo[k]), n);
    }
    g->hi[k] = c;
  }
}

// the modes whose cell costs differ beyond u.dsigma <= 0 (separable fallback of PTM / PTB)
static bool cost_prepass(const Group* g) { return g->have_params && (g->p.df_mode == 3 || g->p.df_mode == 4); }

// full (PTMA warm-start chains): windows of whole chain positions -- each boundary rounded to a multiple of the
// chain count C, so a shard's cells are positions [q0, q1) of every chain
static void chain_windows(Group* g, long n) {
  const int K = (int)g->sh.size();
  const long C = std::max(1L, std::min<long>(g->p.famod_chains, n)), P = (n + C - 1) / C;
  g->q0.assign(K, 0);
  g->q1.assign(K, 0);
  for (int k = 0; k < K; k++) {
    g->q0[k] = k ? g->q1[k - 1] : 0;
    g->q1[k] = (k == K - 1) ? P : std::max(g->q0[k], std::min(P, (g->hi[k] + C / 2) / C));
    g->lo[k] = std::min(n, g->q0[k] * C);
    g->hi[k] = std::min(n, g->q1[k] * C);
  }
}

int group_set_surface(Group* g, long n, const is3d_surface* s) {
  if (!s || n < 0) return g->fail(IS3D_ERR_ARG, "bad surface");
  if (n > 0 && (!s->tau || !s->dat || !s->dax || !s->day || !s->dan || !s->ux || !s->uy || !s->un))
    return g->fail(IS3D_ERR_ARG, "surface field missing");
  g->ncell = n;
  // PTM / PTB: the separable-fallback cells cost 1.4 / 1.8 of a modified one; the prepass on shard 0 knows which
  // cells they are (the tables must be set: otherwise the u.dsigma model)
  std::vector<double> cost;
  if (g->sh.size() > 1 && n > 0 && cost_prepass(g) && is3d_set_surface(g->sh[0], n, s) == IS3D_OK) {
    cost.resize((size_t)n);
    if (is3d_cell_costs(g->sh[0], cost.data()) != IS3D_OK) cost.clear();
  }
  balance(g, n, s->tau, s->dat, s->dax, s->day, s->dan, s->ux, s->uy, s->un, cost.empty() ? nullptr : cost.data());
  g->full = needs_full(g);
  if (g->full) chain_windows(g, n);
  return each_parallel(g, [&](int k) -> int {
    is3d_engine* e = g->sh[k];
    if (g->full) {
      const int rc = is3d_set_surface(e, n, s);
      return rc ? rc : is3d_set_cell_window(e, g->lo[k], g->hi[k]);
    }
    const long o = g->lo[k];
    auto at = [&](const double* f) { return f ? f + o : nullptr; };
    const is3d_surface w{at(s->tau), at(s->x), at(s->y), at(s->eta), at(s->dat), at(s->dax), at(s->day), at(s->dan),
                         at(s->ux), at(s->uy), at(s->un), at(s->E), at(s->T), at(s->P), at(s->pixx), at(s->pixy),
                         at(s->pixn), at(s->piyy), at(s->piyn), at(s->bulkPi), at(s->muB), at(s->nB), at(s->Vx),
                         at(s->Vy), at(s->Vn)};
    const int rc = is3d_set_surface(e, g->hi[k] - o, &w);
    return rc ? rc : is3d_set_cell_window(e, -1, -1);
  });
}

int group_set_surface_device(Group* g, long n, const double* dev_fields) {
  if (n < 0 || (!dev_fields && n > 0)) return g->fail(IS3D_ERR_ARG, "bad device surface");
  // the cost estimate reads the 8 fields it needs back to the host (64 B per cell)
  std::vector<double> h((size_t)8 * std::max(n, 1L));
  const int fidx[8] = {0, 4, 5, 6, 7, 8, 9, 10};   // tau, dat, dax, day, dan, ux, uy, un (is3d_surface order)
  if (hipSetDevice(g->dev[0]) != hipSuccess) return g->fail(IS3D_ERR_DEVICE, "hipSetDevice failed");
  for (int i = 0; i < 8 && n > 0; i++)
    if (hipMemcpy(h.data() + (size_t)i * n, dev_fields + (size_t)fidx[i] * n, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
      return g->fail(IS3D_ERR_DEVICE, "surface read-back failed");
  g->ncell = n;
  std::vector<double> cost;
  if (g->sh.size() > 1 && n > 0 && cost_prepass(g) &&
      is3d_internal_copy_surface(g->sh[0], n, dev_fields, n, g->dev[0], 0) == IS3D_OK) {
    cost.resize((size_t)n);
    if (is3d_cell_costs(g->sh[0], cost.data()) != IS3D_OK) cost.clear();
  }
  balance(g, n, h.data(), h.data() + n, h.data() + 2 * n, h.data() + 3 * n, h.data() + 4 * n, h.data() + 5 * n,
          h.data() + 6 * n, h.data() + 7 * n, cost.empty() ? nullptr : cost.data());
  g->full = needs_full(g);
  if (g->full) chain_windows(g, n);
  return each_parallel(g, [&](int k) -> int {
    is3d_engine* e = g->sh[k];
    const long o = g->full ? 0 : g->lo[k], m = g->full ? n : g->hi[k] - g->lo[k];
    const int rc = is3d_internal_copy_surface(e, m, dev_fields, n, g->dev[0], o);
    if (rc) return rc;
    return g->full ? is3d_set_cell_window(e, g->lo[k], g->hi[k]) : is3d_set_cell_window(e, -1, -1);
  });
}

long group_output_size(const Group* g) { return g->sh.empty() ? -1 : is3d_output_size(g->sh[0]); }

// PTMA warm-start chains split over the shards (see the file comment).  Every pass j of every shard is enqueued
// in reverse shard order, so a shard's pass j waits (event E of its predecessor) for exactly the predecessor's push
// of its pass j - 1 end states, and a shard pushes its pass j end states into its successor's parity-j slot only
// after the successor's pass j (event F), the last reader of that slot (its pass j - 1 read it).  The finishers
// then run in shard order, each handing its final end states (and whether it walked) to the next.
template <class S>
static int launch_split_chains(Group* g, S stream_of) {
  const int K = (int)g->sh.size();
  std::vector<int> act;                 // shards with chain positions, in order
  for (int k = 0; k < K; k++) {
    const int rc = is3d_internal_launch_begin(g->sh[k], g->buf[k], (void*)stream_of(k), g->q0[k], g->q1[k],
                                              act.empty() ? 0 : 1);
    if (rc) return g->shard_fail(k, rc);
    if (g->q1[k] > g->q0[k]) act.push_back(k);
  }
  const int na = (int)act.size();
  const int npass = na ? is3d_internal_chain_npass(g->sh[act[0]]) : 0;
  auto bad = [&](const char* what) { return g->fail(IS3D_ERR_DEVICE, std::string("chain hand-off: ") + what); };
  for (int j = 0; j < npass; j++) {
    for (int i = na - 1; i >= 0; i--) {
      const int k = act[i], kp = i ? act[i - 1] : -1, kn = i + 1 < na ? act[i + 1] : -1;
      if (hipSetDevice(g->dev[k]) != hipSuccess) return bad("hipSetDevice");
      if (kp >= 0 && j > 0 && hipStreamWaitEvent(stream_of(k), g->evE[kp], 0) != hipSuccess) return bad("wait");
      const int rc = is3d_internal_chain_pass(g->sh[k], j);
      if (rc) return g->shard_fail(k, rc);
      if (hipEventRecord(g->evF[k], stream_of(k)) != hipSuccess) return bad("record");
      if (kn >= 0) {
        if (hipStreamWaitEvent(stream_of(k), g->evF[kn], 0) != hipSuccess) return bad("wait");
        if (hipMemcpyPeerAsync(is3d_internal_chain_bnd(g->sh[kn], 0, j & 1), g->dev[kn],
                               is3d_internal_chain_bnd(g->sh[k], 1, j & 1), g->dev[k],
                               is3d_internal_chain_bnd_bytes(g->sh[k]), stream_of(k)) != hipSuccess)
          return bad("hipMemcpyPeerAsync");
        if (hipEventRecord(g->evE[k], stream_of(k)) != hipSuccess) return bad("record");
      }
    }
  }
  for (int i = 0; i < na; i++) {
    const int k = act[i], kp = i ? act[i - 1] : -1, kn = i + 1 < na ? act[i + 1] : -1;
    if (hipSetDevice(g->dev[k]) != hipSuccess) return bad("hipSetDevice");
    if (kp >= 0 && hipStreamWaitEvent(stream_of(k), g->evE[kp], 0) != hipSuccess) return bad("wait");
    const int rc = is3d_internal_chain_end(g->sh[k]);
    if (rc) return g->shard_fail(k, rc);
    if (kn >= 0) {
      if (hipMemcpyPeerAsync(is3d_internal_chain_bnd(g->sh[kn], 0, 2), g->dev[kn], is3d_internal_chain_bnd(g->sh[k], 1, 2),
                             g->dev[k], is3d_internal_chain_bnd_bytes(g->sh[k]), stream_of(k)) != hipSuccess)
        return bad("hipMemcpyPeerAsync");
      if (hipEventRecord(g->evE[k], stream_of(k)) != hipSuccess) return bad("record");
    }
  }
  for (int k = 0; k < K; k++) {
    const int rc = is3d_internal_launch_end(g->sh[k]);
    if (rc) return g->shard_fail(k, rc);
  }
  return IS3D_OK;
}

int group_launch(Group* g, double* dev_out, void* stream) {
  if (!dev_out) return g->fail(IS3D_ERR_ARG, "null output buffer");
  if (stale_split(g)) return g->fail(IS3D_ERR_STATE, kStaleSplit);
  const int K = (int)g->sh.size();
  const long out_n = group_output_size(g);
  if (out_n <= 0) return g->fail(IS3D_ERR_STATE, "species / grids / params not set");
  if ((int)g->buf.size() != K || g->buf_n < out_n) {
    for (int k = 1; k < (int)g->buf.size(); k++) if (g->buf[k]) { (void)hipSetDevice(g->dev[k]); (void)hipFree(g->buf[k]); }
    g->buf.assign(K, nullptr);
    for (int k = 1; k < K; k++) {
      if (hipSetDevice(g->dev[k]) != hipSuccess || hipMalloc(&g->buf[k], out_n * sizeof(double)) != hipSuccess)
        return g->fail(IS3D_ERR_DEVICE, "hipMalloc(shard output) failed");
    }
    if (!g->nccl && K > 1) {
      (void)hipSetDevice(g->dev[0]);
      if (g->scratch) (void)hipFree(g->scratch);
      if (hipMalloc(&g->scratch, out_n * sizeof(double)) != hipSuccess) return g->fail(IS3D_ERR_DEVICE, "hipMalloc(scratch) failed");
    }
    g->buf_n = out_n;
  }
  g->buf[0] = dev_out;
  g->cur0 = (hipStream_t)stream;
  (void)hipSetDevice(g->dev[0]);
  if (hipEventRecord(g->ev0, g->cur0) != hipSuccess) return g->fail(IS3D_ERR_DEVICE, "hipEventRecord failed");
  auto stream_of = [&](int k) { return k ? g->st[k] : g->cur0; };
  const char* dc = std::getenv("IS3D_CHAIN_DIST");
  g->dist_chain = g->full && K > 1 && !(dc && !std::strcmp(dc, "0"));
  if (!g->dist_chain) {
    for (int k = 0; k < K; k++) {
      const int rc = is3d_launch(g->sh[k], g->buf[k], k ? (void*)g->st[k] : stream);
      if (rc) return g->shard_fail(k, rc);
    }
  } else {
    const int rc = launch_split_chains(g, stream_of);
    if (rc) return rc;
  }
  if (g->nccl) {
    if (ncclGroupStart() != ncclSuccess) return g->fail(IS3D_ERR_DEVICE, "ncclGroupStart failed");
    for (int k = 0; k < K; k++) {
      if (ncclAllReduce(g->buf[k], g->buf[k], (size_t)out_n, ncclFloat64, ncclSum, g->comm[k], stream_of(k)) != ncclSuccess) {
        ncclGroupEnd();
        return g->fail(IS3D_ERR_DEVICE, "ncclAllReduce failed");
      }
    }
    if (ncclGroupEnd() != ncclSuccess) return g->fail(IS3D_ERR_DEVICE, "ncclGroupEnd failed");
  } else {
    // shards 1.. in order onto device 0's output: wait for shard k, bring its slab over (peer copy; a repeated
    // device adds in place), add -- a fixed summation order, so repeated runs are bit-identical
    const unsigned nb = (unsigned)std::min<long>((out_n + 255) / 256, 8192);
    for (int k = 1; k < K; k++) {
      (void)hipSetDevice(g->dev[k]);
      if (hipEventRecord(g->done[k], g->st[k]) != hipSuccess) return g->fail(IS3D_ERR_DEVICE, "hipEventRecord failed");
      (void)hipSetDevice(g->dev[0]);
      if (hipStreamWaitEvent(g->cur0, g->done[k], 0) != hipSuccess) return g->fail(IS3D_ERR_DEVICE, "hipStreamWaitEvent failed");
      const double* src = g->buf[k];
      if (g->dev[k] != g->dev[0]) {
        if (hipMemcpyPeerAsync(g->scratch, g->dev[0], g->buf[k], g->dev[k], out_n * sizeof(double), g->cur0) != hipSuccess)
          return g->fail(IS3D_ERR_DEVICE, "hipMemcpyPeerAsync failed");
        src = g->scratch;
      }
      hipLaunchKernelGGL(k_accum, dim3(nb), dim3(256), 0, g->cur0, g->buf[0], src, out_n);
      if (hipGetLastError() != hipSuccess) return g->fail(IS3D_ERR_DEVICE, "k_accum launch failed");
    }
  }
  for (int k = 1; k < K; k++) {     // shard k's stream (nccl: its all-reduce step) enqueued up to here
    (void)hipSetDevice(g->dev[k]);
    if (hipEventRecord(g->done[k], g->st[k]) != hipSuccess) return g->fail(IS3D_ERR_DEVICE, "hipEventRecord failed");
  }
  (void)hipSetDevice(g->dev[0]);
  if (hipEventRecord(g->ev1, g->cur0) != hipSuccess) return g->fail(IS3D_ERR_DEVICE, "hipEventRecord failed");
  g->launched = true;
  return IS3D_OK;
}

int group_finish(Group* g) {
  if (!g->launched) return g->fail(IS3D_ERR_STATE, "nothing launched");
  g->launched = false;
  const int K = (int)g->sh.size();
  int first = IS3D_OK, first_k = 0;
  is3d_stats agg{};
  for (int k = 0; k < K; k++) {
    const int rc = is3d_finish(g->sh[k]);
    if (rc && !first) { first = rc; first_k = k; }
    (void)hipSetDevice(g->dev[k]);
    if (k > 0) (void)hipEventSynchronize(g->done[k]);
    is3d_stats s{};
    is3d_get_stats(g->sh[k], &s);
    agg.cells += s.cells; agg.breakdown += s.breakdown; agg.pl_negative += s.pl_negative;
    agg.recon_fail += s.recon_fail; agg.iterations += s.iterations;
    agg.ms_prepass = std::max(agg.ms_prepass, s.ms_prepass);
    agg.ms_spectra = std::max(agg.ms_spectra, s.ms_spectra);
  }
  (void)hipSetDevice(g->dev[0]);
  if (hipEventSynchronize(g->ev1) != hipSuccess) return g->fail(IS3D_ERR_DEVICE, "group synchronisation failed");
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, g->ev0, g->ev1) == hipSuccess) agg.ms_total = ms;
  if (g->full && !g->dist_chain) {
    // every shard walked the whole PTMA chain and prepared every cell: count that work once (shard 0's, the
    // same solves everywhere)
    is3d_stats s0{};
    is3d_get_stats(g->sh[0], &s0);
    agg.pl_negative = s0.pl_negative; agg.recon_fail = s0.recon_fail; agg.iterations = s0.iterations;
    agg.breakdown = s0.breakdown;
    agg.cells = g->ncell;
  }
  g->stats = agg;
  if (first) return g->shard_fail(first_k, first);
  return IS3D_OK;
}

int group_calculate_spectra(Group* g, double* dN_out) {
  if (!dN_out) return g->fail(IS3D_ERR_ARG, "null output");
  const long n = group_output_size(g);
  if (n <= 0) return g->fail(IS3D_ERR_STATE, "species / grids / params not set");
  (void)hipSetDevice(g->dev[0]);
  if (g->out_n < n) {
    if (g->d_out) (void)hipFree(g->d_out);
    g->d_out = nullptr;
    if (hipMalloc(&g->d_out, n * sizeof(double)) != hipSuccess) return g->fail(IS3D_ERR_DEVICE, "hipMalloc(output) failed");
    g->out_n = n;
  }
  int rc = group_launch(g, g->d_out, nullptr);
  if (!rc) rc = group_finish(g);
  if (rc) return rc;
  (void)hipSetDevice(g->dev[0]);
  if (hipMemcpy(dN_out, g->d_out, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    return g->fail(IS3D_ERR_DEVICE, "spectra download failed");
  return IS3D_OK;
}

int group_calculate_dN_dX(Group* g, double* tau, double* r, double* phi) {
  if (!tau || !r || !phi) return g->fail(IS3D_ERR_ARG, "null output");
  if (!g->have_bins || g->np <= 0) return g->fail(IS3D_ERR_STATE, "species / spacetime bins not set");
  const int K = (int)g->sh.size();
  if (K > 1 && g->bins.threads > 0)
    return g->fail(IS3D_ERR_UNSUPPORTED, "spacetime threads > 0 (the reference's thread-slice carry) runs on one device");
  if (stale_split(g)) return g->fail(IS3D_ERR_STATE, kStaleSplit);
  if (g->full && K > 1)
    return g->fail(IS3D_ERR_UNSUPPORTED, "calculate_spectra error: no spacetime distribution routine for famod yet");
  const long nt = (long)g->np * g->bins.tau_bins, nr = (long)g->np * g->bins.r_bins, nph = (long)g->np * g->bins.phip_bins;
  std::vector<std::vector<double>> part(K, std::vector<double>((size_t)(nt + nr + nph), 0.0));
  const int rc = each_parallel(g, [&](int k) -> int {
    double* b = part[k].data();
    return is3d_calculate_dN_dX(g->sh[k], b, b + nt, b + nt + nr);
  });
  if (rc) return rc;
  // the binned, width-normalised distributions are sums over cells: add the shards in order
  for (long i = 0; i < nt + nr + nph; i++) {
    double a = 0.0;
    for (int k = 0; k < K; k++) a += part[k][i];
    (i < nt ? tau[i] : i < nt + nr ? r[i - nt] : phi[i - nt - nr]) = a;
  }
  is3d_stats agg{};
  for (int k = 0; k < K; k++) {
    is3d_stats s{};
    is3d_get_stats(g->sh[k], &s);
    agg.cells += s.cells;
    agg.ms_prepass = std::max(agg.ms_prepass, s.ms_prepass);
    agg.ms_spectra = std::max(agg.ms_spectra, s.ms_spectra);
    agg.ms_total = std::max(agg.ms_total, s.ms_total);
  }
  g->stats = agg;
  return IS3D_OK;
}

int group_get_cell_yields(const Group* g, double* out) {
  if (!out) return IS3D_ERR_ARG;
  const int K = (int)g->sh.size();
  const long n = g->ncell;
  for (int k = 0; k < K; k++) {
    const long m = g->hi[k] - g->lo[k];
    std::vector<double> y((size_t)g->np * std::max(m, 1L));
    const int rc = is3d_get_cell_yields(g->sh[k], y.data());
    if (rc) return rc;
    for (int s = 0; s < g->np; s++)
      std::copy(y.begin() + (size_t)s * m, y.begin() + (size_t)(s + 1) * m, out + (size_t)s * n + g->lo[k]);
  }
  return IS3D_OK;
}

int group_get_stats(const Group* g, is3d_stats* out) {
  *out = g->stats;
  return IS3D_OK;
}

int group_evaluate_df_coefficients(Group* g, double T, double muB, double E, double P, double bulkPi, double* out15) {
  const int rc = is3d_evaluate_df_coefficients(g->sh[0], T, muB, E, P, bulkPi, out15);
  return rc ? g->shard_fail(0, rc) : IS3D_OK;
}

int group_total_yield(Group* g, const double* plasma, double y_cut, double* n_total, double* densities) {
  if (!plasma || !n_total) return g->fail(IS3D_ERR_ARG, "null argument");
  if (stale_split(g)) return g->fail(IS3D_ERR_STATE, kStaleSplit);
  const int K = (int)g->sh.size();
  std::vector<double> nt(K, 0.0);
  const int rc = each_parallel(g, [&](int k) -> int {
    if (g->full) {   // every shard holds the whole surface: only shard 0 counts it
      if (k) return IS3D_OK;
      return is3d_total_yield(g->sh[0], plasma, y_cut, &nt[0], densities);
    }
    return is3d_total_yield(g->sh[k], plasma, y_cut, &nt[k], k ? nullptr : densities);
  });
  if (rc) return rc;
  double s = 0.0;
  for (int k = 0; k < K; k++) s += nt[k];
  *n_total = s;
  return IS3D_OK;
}

int group_get_jonah_table(const Group* g, double* l2, double* z, double* bp, double* bpmax) {
  return is3d_get_jonah_table(g->sh[0], l2, z, bp, bpmax);
}

}  // namespace is3d

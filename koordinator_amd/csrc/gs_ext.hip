// gs_ext.hip — Reservation + DeviceShare kernels for one extension pod (see gs_ext.h).
//
// Reference: deviceshare/plugin.go:272-322 (Filter), deviceshare/scoring.go:34-89,186-308 (Score),
// deviceshare/device_allocator.go:99-163,397-467,513-536 (Allocate / score), devicehandler_gpu.go:38-85 (desired
// per-instance request), reservation/transformer.go:50-292 (restore), reservation/plugin.go:311-496 (Filter, fitsNode),
// reservation/nominator.go:140-190 + scoring.go:42-203 (nomination, PreScore, Score),
// [upstream] pluginhelper.DefaultNormalizeScore, schedule_one.go selectHost.
#include <hip/hip_runtime.h>

#include "gs_eval_dev.h"
#include "gs_ext.h"

namespace gs {
namespace {

constexpr int64_t kMaxNodeScore = 100;

__device__ __forceinline__ int64_t ds_least(int64_t req, int64_t cap) {
  return (cap == 0 || req > cap) ? 0 : (cap - req) * kMaxNodeScore / cap;
}
__device__ __forceinline__ int64_t ds_most(int64_t req, int64_t cap) {
  if (cap == 0) return 0;
  if (req > cap) req = cap;
  return req * kMaxNodeScore / cap;
}

// GPUHandler.CalcDesiredRequestsAndCount: per-instance request (all three keys after fillGPUTotalMem) and count;
// false = Prepare fails (no GPU minors / no healthy GPU)
__device__ __forceinline__ bool gpu_desired(const DevNode& d, const ExtPod& p, int64_t inst[3], uint32_t* mask,
                                            int64_t* count) {
  if (d.num_gpus <= 0) return false;
  int64_t total_mem = -1;
  for (int g = 0; g < d.num_gpus; ++g) {
    if (d.g[g].total[0] | d.g[g].total[1] | d.g[g].total[2]) { total_mem = d.g[g].total[2]; break; }
  }
  if (total_mem < 0) return false;
  int64_t core = p.gpu_req[0], ratio = p.gpu_req[1], mem = p.gpu_req[2];
  if (p.gpu_mask & 4u) ratio = (int64_t)((double)mem / (double)total_mem * 100.0);   // memoryBytesToRatio
  else mem = ratio * total_mem / 100;                                                   // memoryRatioToBytes
  uint32_t m = p.gpu_mask | 6u;
  int64_t n = 1;
  if (ratio > 100 && ratio % 100 == 0) {
    n = ratio / 100;
    core /= n; mem /= n; ratio /= n;
    m = 7u;
  }
  inst[0] = core; inst[1] = ratio; inst[2] = mem;
  *mask = m;
  *count = n;
  return true;
}

__device__ __forceinline__ bool fits_inst(const int64_t inst[3], uint32_t mask, const DevGpu& g) {
  for (int r = 0; r < 3; ++r)
    if ((mask >> r & 1u) && inst[r] > g.free[r]) return false;
  return true;
}

// one node: GPU Fit scalars, DeviceShare Filter and raw Score
// [upstream] fitsRequest over the pod's GPU-name / registered extended scalars (every node, matched ones included)
__device__ __forceinline__ bool fit_names_ok(const DevNode& d, const ExtPod& p) {
  for (int n = 0; n < EXT_FIT_NAMES; ++n)
    if ((p.gpu_names >> n & 1u) && p.gpu_name_req[n] > d.fit_free[n]) return false;
  return true;
}

// aff: the node's NUMA affinity (0x10 | zone-slot mask; 0 = none): filterNodeDevice keeps only the minors whose
// Topology is on it (device_allocator.go:139-163)
__device__ __forceinline__ bool on_aff(const DevGpu& x, uint32_t aff) {
  return !(aff & 0x10u) || (x.zone >= 0 && (aff >> x.zone & 1u));
}

__device__ __forceinline__ void eval_device(const DevNode& d, const ExtPod& p, bool* ok, int32_t* raw,
                                            uint32_t aff = 0) {
  *ok = true;
  *raw = 0;
  if (!fit_names_ok(d, p)) { *ok = false; return; }
  if (!d.has_device || !p.gpu_mask) return;   // no Device object / no GPU request: DeviceShare passes, scores 0
  int64_t inst[3];
  uint32_t mask;
  int64_t count;
  if (!gpu_desired(d, p, inst, &mask, &count)) { *ok = false; return; }
  // nodeDevice.filter: a node whose GPUs are all fully used drops the type
  bool all_zero = true;
  for (int g = 0; g < d.num_gpus; ++g) all_zero &= !(d.g[g].free[0] | d.g[g].free[1] | d.g[g].free[2]);
  int64_t ok_n = 0, tot[3] = {0, 0, 0}, fr[3] = {0, 0, 0};
  if (!all_zero) {
    for (int g = 0; g < d.num_gpus; ++g) {
      const DevGpu& x = d.g[g];
      if (!x.has_info || !on_aff(x, aff)) continue;
      for (int r = 0; r < 3; ++r) { tot[r] += x.total[r]; fr[r] += x.free[r]; }
      if (!(x.free[0] | x.free[1] | x.free[2])) continue;
      if (fits_inst(inst, mask, x)) ++ok_n;
    }
  }
  if (ok_n < count) { *ok = false; return; }
  // allocator.score -> scoreNode (summed totals / frees of the candidate minors)
  int64_t ns = 0, ws = 0;
  for (int r = 0; r < 3; ++r) {
    if (!p.dev_w[r] || tot[r] == 0) continue;
    int64_t rq = tot[r];
    if (tot[r] >= fr[r]) rq = tot[r] - fr[r] + ((mask >> r & 1u) ? inst[r] : 0);
    ns += (p.dev_most ? ds_most(rq, tot[r]) : ds_least(rq, tot[r])) * p.dev_w[r];
    ws += p.dev_w[r];
  }
  *raw = ws ? (int32_t)(ns / ws) : 0;
}

constexpr int ACC_WORDS_N = 8;   // (ACC_* below)
__global__ __launch_bounds__(256) void ext_nodes_kernel(const DevNode* __restrict__ dev, const int16_t* __restrict__ S,
                                                         uint32_t n0, uint32_t n1, const ExtPod* __restrict__ pp,
                                                         int32_t* tot, int16_t* ds, int16_t* rs, int32_t* acc) {
  // the select accumulators start from zero (ACC_PREF: -1, no preferred node unless ext_matched_kernel finds one)
  if (blockIdx.x == 0 && threadIdx.x < ACC_WORDS_N) acc[threadIdx.x] = threadIdx.x == 6 ? -1 : 0;
  const uint32_t i = n0 + blockIdx.x * 256 + threadIdx.x;
  if (i >= n1) return;
  const ExtPod& p = *pp;
  int32_t t = S[i - n0];
  int32_t raw = 0;
  if (t >= 0 && (p.gpu_mask || p.gpu_names)) {
    bool ok;
    eval_device(dev[i], p, &ok, &raw);
    if (!ok) t = -1;
  }
  if (p.required) t = -1;       // reservation affinity: only nodes with a matched reservation (ext_matched_kernel)
  tot[i - n0] = t;
  ds[i - n0] = (int16_t)(t >= 0 ? raw : 0);
  rs[i - n0] = 0;
}

// DeviceShare GetPodTopologyHints (topology_hint.go:108-214) on one node with nz NUMA zones, packed as GH_* (gs_numa_dev.h).
// IterateBitMasks over the zones holding GPUs with a Topology visits exactly the positions whose mask lies within that
// zone set, in position order. *bad: a GPU on a NUMA node outside the node's zones.
__device__ uint32_t gpu_hint_word(const DevNode& d, const ExtPod& p, int nz, bool* bad) {
  if (!d.has_device || !p.gpu_mask) return 0;
  uint32_t zs = 0;   // numaTopology.nodes
  for (int g = 0; g < d.num_gpus; ++g) {
    if (!d.g[g].has_info) continue;
    if (d.g[g].zone == GZ_FOREIGN) *bad = true;
    if (d.g[g].zone >= 0) zs |= 1u << d.g[g].zone;
  }
  int64_t inst[3];
  uint32_t mask;
  int64_t count;
  if (!zs || !gpu_desired(d, p, inst, &mask, &count)) return 0;   // no mask visited / Prepare fails: no hints
  bool all_zero = true;
  for (int g = 0; g < d.num_gpus; ++g) all_zero &= !(d.g[g].free[0] | d.g[g].free[1] | d.g[g].free[2]);
  const uint32_t valid = ord_valid(nz);
  int minsz = -1;
  uint32_t list = 0;
  for (int mi = 0; mi < 15; ++mi) {
    const uint32_t mk = ord_mask(mi);
    if (!(valid >> mi & 1u) || (mk & ~zs)) continue;
    int64_t total = 0, ok_n = 0;   // calcTotalDevicesByNUMA; the allocation within the mask
    for (int g = 0; g < d.num_gpus; ++g) {
      const DevGpu& x = d.g[g];
      if (!x.has_info || x.zone < 0 || !(mk >> x.zone & 1u)) continue;
      ++total;
      if (!all_zero && (x.free[0] | x.free[1] | x.free[2]) && fits_inst(inst, mask, x)) ++ok_n;
    }
    if (total < count) continue;
    if (minsz < 0) minsz = __popc(zs);
    if (__popc(mk) < minsz) minsz = __popc(mk);
    if (ok_n >= count) list |= 1u << mi;
  }
  if (minsz < 0) return 0;   // minAffinitySize nil: an empty map
  return list | ((uint32_t)minsz << GH_MIN_SHIFT) | ((uint32_t)__popc(mask) << GH_R_SHIFT);
}

// fitsNode (plugin.go:444-496), preemptible = 0: number of insufficient resources
__device__ int fits_node(const ExtPod& p, const ExtRec& rc, const ExtRes* r) {
  int bad = 0;
  if (rc.restored_pods - rc.nres + 1 > rc.allowed_pods) ++bad;
  const uint32_t scalars = p.pod_mask & GS_SCALAR_RES_MASK;
  if (!p.pod_req[0] && !p.pod_req[1] && !p.pod_req[2] && !scalars) return bad;
  for (int s = 0; s < 7; ++s) {
    if (s >= 3 && !(scalars >> s & 1u)) continue;
    const int64_t rem = r ? r->alloc[s] - r->allocated[s] : 0;
    const int64_t avail = rc.allocatable[s] - (rc.pod_requested[s] - rem - rc.r_allocated[s]);
    if (p.pod_req[s] > avail) ++bad;
  }
  return bad;
}

// filterWithReservations over one reservation (plugin.go:377-440)
__device__ bool reservation_fits(const ExtPod& p, const ExtRec& rc, const ExtRes& r) {
  if (!(r.names & p.pod_mask)) return false;
  const bool node_fits = fits_node(p, rc, &r) == 0;
  if (r.policy == GS_RSV_POLICY_DEFAULT || r.policy == GS_RSV_POLICY_ALIGNED) return node_fits;
  if (r.policy == GS_RSV_POLICY_RESTRICTED) {
    if (!node_fits) return false;
    for (int s = 0; s < 7; ++s)
      if ((p.pod_mask >> s & 1u) && (r.names >> s & 1u) && p.pod_req[s] > r.remained_nn[s]) return false;
    return true;
  }
  return false;
}

__device__ __forceinline__ int64_t milli(int s, int64_t v) { return s == 0 ? v : v * 1000; }

// scoreReservation (scoring.go:183-203) with allocated = Allocated
__device__ int64_t score_reservation(const ExtPod& p, const ExtRes& r) {
  int64_t s = 0, w = 0;
  for (int k = 0; k < 7; ++k) {
    if (!(r.alloc_mask >> k & 1u) || r.alloc[k] == 0) continue;
    ++w;
    const int64_t req = ((p.pod_mask >> k & 1u) ? p.pod_req[k] : 0) + ((r.allocated_mask >> k & 1u) ? r.allocated[k] : 0);
    if (req <= r.alloc[k]) s += kMaxNodeScore * milli(k, req) / milli(k, r.alloc[k]);
  }
  return w ? s / w : 0;
}

constexpr int SEL_BLOCK = 256;
constexpr int SEL_PER = 4;                       // nodes per thread in the select passes
constexpr int SEL_SPAN = SEL_BLOCK * SEL_PER;     // nodes per block (a contiguous range: the ties pass relies on it)
enum { ACC_DS = 0, ACC_RS = 1, ACC_FEAS = 2, ACC_MAX = 3, ACC_DONE = 4, ACC_TIES = 5, ACC_PREF = 6, ACC_ERR = 7,
       ACC_WORDS = 8 };
static_assert(ACC_WORDS == ACC_WORDS_N && ACC_PREF == 6, "accumulator layout (ext_nodes_kernel resets it)");

// GPU pods on NUMA-policy nodes: the pair again with DeviceShare as the second hint provider (the eval pass merged
// NodeNUMAResource's hints alone), then Fit's GPU scalars and DeviceShare Filter / raw Score within the affinity
// (the topology manager's Admit -> DeviceShare.Allocate, topology_hint.go:57-106; Filter / Score, plugin.go:272-322,
// scoring.go:34-89, read the same store entry).
__global__ __launch_bounds__(256) void ext_numa_kernel(MirrorView m, const PodVec* __restrict__ pods, Profile pf,
                                                       int prod_cols, const DevNode* __restrict__ dev,
                                                       const ExtPod* __restrict__ pp, const uint32_t* __restrict__ idx,
                                                       uint32_t nidx, uint32_t n0, int32_t* tot, int16_t* ds,
                                                       uint8_t* aff, int32_t* acc) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= nidx) return;
  const ExtPod& p = *pp;
  const uint32_t i = idx[t];
  Row r;
  load_row(m, i, prod_cols != 0, true, r);
  for (int s = 3; s < 7; ++s) r.free[s] = m.c64(C_FREE_CPU + s)[i];
  const int nz = (r.nr.nflags >> NF_ZONES_SHIFT) & 7;
  bool bad = false, over = false;
  const uint32_t gh = gpu_hint_word(dev[i], p, nz, &bad);
  const PairOut o = eval_pair<false, true, true, false, false, true>(r, pods[0], pf, m, nullptr, gh, &over);
  int32_t t_sc = total_score(o, pf);
  int32_t raw = 0;
  if (t_sc >= 0 && (p.gpu_mask || p.gpu_names)) {
    bool ok;
    eval_device(dev[i], p, &ok, &raw, o.aff);
    if (!ok) t_sc = -1;
  }
  if (p.required) t_sc = -1;
  tot[i - n0] = t_sc;
  ds[i - n0] = (int16_t)(t_sc >= 0 ? raw : 0);
  aff[i - n0] = (uint8_t)(o.code ? 0u : o.aff);
  if (bad || over) atomicOr(&acc[ACC_ERR], (bad ? 1 : 0) | (over ? 2 : 0));
}

// The pod's end. NodeNUMAResource Reserve (plugin.go:375-422) of the selected node: Allocate along its Filter-time
// affinity; then the result and the nominations into pinned host memory.
__global__ __launch_bounds__(64) void ext_finish_kernel(MirrorView m, const PodVec* __restrict__ pods, Profile pf,
                                                        int prod_cols, const uint8_t* __restrict__ aff, uint32_t n0,
                                                        int numa, const ExtOut* __restrict__ dout,
                                                        const int32_t* __restrict__ nom, int nrec, ExtOut* hout,
                                                        int32_t* hnom) {
  for (int k = threadIdx.x; k < nrec; k += 64) hnom[k] = nom[k];
  if (threadIdx.x == 0) {
    ExtOut o = *dout;
    if (numa && o.node >= 0) {
      Row r;
      load_row(m, (uint32_t)o.node, prod_cols != 0, true, r);
      for (int s = 3; s < 7; ++s) r.free[s] = m.c64(C_FREE_CPU + s)[o.node];
      const NumaOut no = numa_eval<true>(r.nr, pods[0], pf, SlotsLds{r, m}, true, false, aff[o.node - n0]);
      o.nflags = no.flags | (no.reason ? PL_RESERVE_FAILED : 0u);
      o.zkeys = no.zkeys;
      for (int z = 0; z < 4; ++z) { o.zcpu[z] = no.zcpu[z]; o.zmem[z] = no.zmem[z]; }
      o.aff = no.aff;
    }
    *hout = o;
  }
  __threadfence_system();
}

// one matched node (record k): the restored row re-evaluated, Reservation Filter, NominateReservation, raw Score.
// Runs after ext_nodes / ext_numa and has the last word on its node: the whole Filter chain over the restored NodeInfo
// (Fit, LoadAware, NodeNUMAResource — with DeviceShare as the second hint provider for a GPU pod on a NUMA-policy
// node — and DeviceShare's Filter / raw Score within the affinity; the reservations modelled hold no devices, so
// DeviceShare's view of the node is not restored: deviceshare/reservation.go:133-162 keeps device-holding ones only),
// and the Filter-time affinity of a policy node (the unrestored eval pass may have stopped before NodeNUMAResource).
__device__ __forceinline__ void matched_one(const MirrorView& m, const PodVec* __restrict__ pods, const Profile& pf,
                                            int prod_cols, const DevNode* __restrict__ dev, const ExtPod& p,
                                            const ExtRec* __restrict__ recs,
                                            const ExtRes* __restrict__ res, int k, int32_t* tot, int16_t* ds,
                                            int16_t* rs, int32_t* nominated, uint8_t* aff, uint32_t n0, int32_t* acc) {
  const ExtRec& rc = recs[k];
  const uint32_t i = rc.node;
  // the restored NodeInfo of the pod (BeforePreFilter): the mirror row plus the matched restore deltas
  Row r;
  const bool numa_on = (pf.enabled & 0x30u) != 0;
  load_row(m, i, prod_cols != 0, numa_on, r);
  for (int s = 3; s < 7; ++s) r.free[s] = m.c64(C_FREE_CPU + s)[i];
  for (int s = 0; s < 7; ++s) r.free[s] += rc.dfree[s];
  r.nzfree[0] += rc.dnz[0];
  r.nzfree[1] += rc.dnz[1];
  r.free_pods += rc.dpods;
  const bool pol = numa_on && ((r.nr.nflags >> NF_POLICY_SHIFT) & 3u);
  PairOut o;
  if (pol && p.gpu_mask) {   // DeviceShare as the topology manager's second hint provider (as ext_numa_kernel)
    bool bad = false, over = false;
    const int nz = (r.nr.nflags >> NF_ZONES_SHIFT) & 7;
    const uint32_t gh = gpu_hint_word(dev[i], p, nz, &bad);
    o = eval_pair<false, true, true, false, false, true>(r, pods[0], pf, m, nullptr, gh, &over);
    if (bad || over) atomicOr(&acc[ACC_ERR], (bad ? 1 : 0) | (over ? 2 : 0));
  } else {
    o = eval_pair<false, true>(r, pods[0], pf, m);
  }
  int32_t t = total_score(o, pf);
  int32_t raw = 0;
  if (t >= 0 && (p.gpu_mask || p.gpu_names)) {   // Fit's GPU-name scalars (not restored) and DeviceShare's Filter
    bool ok;
    eval_device(dev[i], p, &ok, &raw, pol ? o.aff : 0u);
    if (!ok) t = -1;
  }
  if (pol) aff[i - n0] = (uint8_t)(o.code ? 0u : o.aff);
  // Reservation Filter: a required pod needs a satisfying matched reservation (filterWithReservations)
  if (t >= 0 && p.required) {
    bool any = false;
    for (int j = 0; j < rc.nres && !any; ++j) any = reservation_fits(p, rc, res[rc.first + j]);
    if (!any) t = -1;
  }
  // NominateReservation (nominator.go:140-190). RunReservationFilterPlugins also runs DeviceShare's FilterReservation,
  // which fails for a device pod on every reservation without device allocations (deviceshare/plugin.go:338-350): a
  // GPU pod nominates none
  int nom = -1;
  if (t >= 0 && !p.gpu_mask) {
    int64_t best_order = INT64_MAX;
    for (int j = 0; j < rc.nres; ++j) {
      const ExtRes& x = res[rc.first + j];
      if (x.skip || !reservation_fits(p, rc, x)) continue;
      if (x.order != 0 && best_order > x.order) { best_order = x.order; nom = j; }
    }
    if (nom < 0) {
      int64_t bs = INT64_MIN;
      for (int j = 0; j < rc.nres; ++j) {
        const ExtRes& x = res[rc.first + j];
        if (x.skip || !reservation_fits(p, rc, x)) continue;
        const int64_t s = score_reservation(p, x);
        if (s > bs) { bs = s; nom = j; }
      }
    }
  }
  tot[i] = t;
  ds[i] = (int16_t)(t >= 0 ? raw : 0);
  rs[i] = (int16_t)((t >= 0 && nom >= 0) ? score_reservation(p, res[rc.first + nom]) : 0);
  nominated[k] = nom;
}

// One workgroup over the matched records, then PreScore's preferred node: the first feasible matched node (node
// order) with the lowest reservation order (findMostPreferredReservationByOrder, scoring.go:89-99) -> acc[ACC_PREF].
__global__ __launch_bounds__(SEL_BLOCK) void ext_matched_kernel(MirrorView m, const PodVec* __restrict__ pods,
                                                                Profile pf, int prod_cols, const DevNode* __restrict__ dev,
                                                                const ExtPod* __restrict__ pp,
                                                                const ExtRec* __restrict__ recs,
                                                                const ExtRes* __restrict__ res, int nrec, int32_t* tot,
                                                                int16_t* ds, int16_t* rs, int32_t* nominated,
                                                                uint8_t* aff, uint32_t n0, int32_t* acc) {
  __shared__ int64_t so_sh[SEL_BLOCK];
  __shared__ int32_t node_sh[SEL_BLOCK];
  const ExtPod& p = *pp;
  int64_t so = INT64_MAX;
  int32_t pn = -1;
  for (int k = threadIdx.x; k < nrec; k += SEL_BLOCK) {
    matched_one(m, pods, pf, prod_cols, dev, p, recs, res, k, tot, ds, rs, nominated, aff, n0, acc);
    const ExtRec& rc = recs[k];
    if (tot[rc.node] >= 0 && rc.order_min != INT64_MAX && rc.order_min != 0 &&
        (rc.order_min < so || (rc.order_min == so && (int32_t)rc.node < pn))) {
      so = rc.order_min;
      pn = (int32_t)rc.node;
    }
  }
  so_sh[threadIdx.x] = so;
  node_sh[threadIdx.x] = pn;
  __syncthreads();
  for (int o = SEL_BLOCK / 2; o > 0; o >>= 1) {
    if (threadIdx.x < (unsigned)o) {
      const int64_t a = so_sh[threadIdx.x], b = so_sh[threadIdx.x + o];
      const int32_t na = node_sh[threadIdx.x], nb = node_sh[threadIdx.x + o];
      if (b < a || (b == a && nb >= 0 && (na < 0 || nb < na))) { so_sh[threadIdx.x] = b; node_sh[threadIdx.x] = nb; }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) acc[ACC_PREF] = p.rs_on ? node_sh[0] : -1;
}

// ---- normalizing select over the whole row, in four grid passes (coalesced; no grid-wide barrier):
//   ext_acc_kernel    per-block max of the DeviceShare / Reservation raw scores (PreScore's preferred node counted at
//                     mostPreferredScore) and the feasible count -> global atomics
//   ext_total_kernel  weighted totals T[j] with both DefaultNormalizeScore passes, per-block max -> atomicMax
//   ext_ties_kernel   per-block tie counts at the max (blocks cover contiguous node ranges); the last block to finish
//                     scans the block counts, finds the block of the j*-th tie (selectHost) and the node in it
// A block covers SEL_SPAN nodes, SEL_PER per thread in SEL_BLOCK-wide coalesced chunks: a quarter of the blocks and of
// the same-address atomics of one node per thread (the three passes 27.6 -> 18.8 us per pod at 100k nodes; 2 and 8
// per thread measured 20.6 and 22.5 us, profiles/r06_c5_select_span.txt)

__device__ __forceinline__ int32_t block_max_i32(int32_t v, int32_t* sh) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  int32_t m = sh[0];
  for (int i = 1; i < SEL_BLOCK / 64; ++i) m = max(m, sh[i]);
  __syncthreads();
  return m;
}
__device__ __forceinline__ int32_t block_sum_i32(int32_t v, int32_t* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  int32_t m = 0;
  for (int i = 0; i < SEL_BLOCK / 64; ++i) m += sh[i];
  __syncthreads();
  return m;
}

__global__ __launch_bounds__(SEL_BLOCK) void ext_acc_kernel(const int32_t* __restrict__ tot,
                                                            const int16_t* __restrict__ ds,
                                                            const int16_t* __restrict__ rs,
                                                            const ExtRec* __restrict__ recs, uint32_t n0, uint32_t len,
                                                            const ExtPod* __restrict__ pp, int32_t* acc) {
  __shared__ int32_t sh[SEL_BLOCK / 64];
  const int32_t pref = acc[ACC_PREF];
  int32_t f = 0, d = 0, r = 0;
#pragma unroll
  for (int q = 0; q < SEL_PER; ++q) {
    const uint32_t j = blockIdx.x * SEL_SPAN + q * SEL_BLOCK + threadIdx.x;
    if (j < len && tot[j] >= 0) {
      f += 1;
      d = max(d, (int32_t)ds[j]);
      r = max(r, (int32_t)(j + n0) == pref ? 1000 : (int32_t)rs[j]);
    }
  }
  d = block_max_i32(d, sh);
  r = block_max_i32(r, sh);
  f = block_sum_i32(f, sh);
  if (threadIdx.x == 0) {
    if (d) atomicMax(&acc[ACC_DS], d);
    if (r) atomicMax(&acc[ACC_RS], r);
    if (f) atomicAdd(&acc[ACC_FEAS], f);
  }
}

__global__ __launch_bounds__(SEL_BLOCK) void ext_total_kernel(const int32_t* __restrict__ tot,
                                                              const int16_t* __restrict__ ds,
                                                              const int16_t* __restrict__ rs,
                                                              const ExtRec* __restrict__ recs, uint32_t n0, uint32_t len,
                                                              const ExtPod* __restrict__ pp, int32_t* T, int32_t* acc) {
  __shared__ int32_t sh[SEL_BLOCK / 64];
  const ExtPod& p = *pp;
  const int32_t pref_sh = acc[ACC_PREF];
  const int64_t MDS = acc[ACC_DS], MRS = acc[ACC_RS];
  int32_t tm = -1;
#pragma unroll
  for (int q = 0; q < SEL_PER; ++q) {
    const uint32_t j = blockIdx.x * SEL_SPAN + q * SEL_BLOCK + threadIdx.x;
    int32_t t = -1;
    if (j < len && tot[j] >= 0) {
      int64_t x = tot[j];
      if (p.ds_on) x += (MDS ? kMaxNodeScore * ds[j] / MDS : (int64_t)ds[j]) * p.w_ds;
      if (p.rs_on) {
        const int64_t r = (int32_t)(j + n0) == pref_sh ? 1000 : rs[j];
        x += (MRS ? kMaxNodeScore * r / MRS : r) * p.w_rs;
      }
      t = (int32_t)x;
    }
    if (j < len) T[j] = t;
    tm = max(tm, t);
  }
  const int32_t m = block_max_i32(tm, sh);
  if (threadIdx.x == 0 && m >= 0) atomicMax(&acc[ACC_MAX], m + 1);
}

__global__ __launch_bounds__(SEL_BLOCK) void ext_ties_kernel(const int32_t* __restrict__ T,
                                                             const int16_t* __restrict__ ds,
                                                             const int16_t* __restrict__ rs, uint32_t n0, uint32_t len,
                                                             const ExtPod* __restrict__ pp, uint64_t seed, int32_t* acc,
                                                             int32_t* bcnt, ExtOut* out) {
  __shared__ int32_t sh[SEL_BLOCK / 64];
  __shared__ int32_t last;
  __shared__ int64_t jstar_sh;
  __shared__ int32_t found_block, found_rank;
  const ExtPod& p = *pp;
  const int32_t M = acc[ACC_MAX] - 1;
  int32_t mine_ties = 0;
#pragma unroll
  for (int q = 0; q < SEL_PER; ++q) {
    const uint32_t j = blockIdx.x * SEL_SPAN + q * SEL_BLOCK + threadIdx.x;
    mine_ties += (M >= 0 && j < len && T[j] == M) ? 1 : 0;
  }
  const int32_t c = block_sum_i32(mine_ties, sh);
  if (threadIdx.x == 0) {
    bcnt[blockIdx.x] = c;
    __threadfence();
    last = atomicAdd(&acc[ACC_DONE], 1) == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  const int32_t F = __atomic_load_n(&acc[ACC_FEAS], __ATOMIC_RELAXED);
  const int32_t pref = acc[ACC_PREF];
  const uint32_t err = (uint32_t)__atomic_load_n(&acc[ACC_ERR], __ATOMIC_RELAXED);
  if (M < 0) {
    if (threadIdx.x == 0) {
      ExtOut o{};
      o.node = -1; o.feasible = (uint32_t)F; o.rec = -1; o.pref_node = pref; o.err = err;
      *out = o;
    }
    return;
  }
  // the last block: thread t owns block counts [t*per, (t+1)*per); a block scan gives every range its tie offset
  const uint32_t nb = gridDim.x, per = (nb + SEL_BLOCK - 1) / SEL_BLOCK;
  const uint32_t b0 = min(nb, threadIdx.x * per), b1 = min(nb, b0 + per);
  int32_t mine = 0;
  for (uint32_t b = b0; b < b1; ++b) mine += __atomic_load_n(&bcnt[b], __ATOMIC_RELAXED);
  const int incl = wave_incl_scan(mine);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) sh[w] = incl;
  __syncthreads();
  int32_t before = incl - mine, ties = 0;
  for (int i = 0; i < SEL_BLOCK / 64; ++i) {
    if (i < w) before += sh[i];
    ties += sh[i];
  }
  if (threadIdx.x == 0) {
    jstar_sh = tiebreak_position(seed, p.seq, ties);
    acc[ACC_TIES] = ties;
  }
  __syncthreads();
  const int64_t jstar = jstar_sh;
  if (jstar > before && jstar <= before + mine) {
    int64_t cum = before;
    for (uint32_t b = b0; b < b1; ++b) {
      const int32_t cb = __atomic_load_n(&bcnt[b], __ATOMIC_RELAXED);
      if (jstar <= cum + cb) { found_block = (int32_t)b; found_rank = (int32_t)(jstar - cum); break; }
      cum += cb;
    }
  }
  __syncthreads();
  // the found block's range in node order, one SEL_BLOCK chunk at a time (seen: the ties of its earlier chunks)
  int32_t seen = 0;
  for (int q = 0; q < SEL_PER && seen < found_rank; ++q) {
    const uint32_t jj = (uint32_t)found_block * SEL_SPAN + q * SEL_BLOCK + threadIdx.x;
    const int is_tie = (jj < len && __atomic_load_n(&T[jj], __ATOMIC_RELAXED) == M) ? 1 : 0;
    const int tincl = wave_incl_scan(is_tie);
    if ((threadIdx.x & 63) == 63) sh[w] = tincl;
    __syncthreads();
    int rank = seen + tincl, chunk = 0;
    for (int i = 0; i < SEL_BLOCK / 64; ++i) {
      if (i < w) rank += sh[i];
      chunk += sh[i];
    }
    seen += chunk;
    __syncthreads();   // (sh is rewritten by the next chunk)
    if (is_tie && rank == found_rank) {
      const int32_t node = (int32_t)(jj + n0);
      const int64_t MDS = acc[ACC_DS], MRS = acc[ACC_RS];
      const int64_t dsn = MDS ? kMaxNodeScore * ds[jj] / MDS : ds[jj];
      const int64_t rr = node == pref ? 1000 : rs[jj];
      const int64_t rsn = MRS ? kMaxNodeScore * rr / MRS : rr;
      ExtOut o{};
      o.node = node; o.feasible = (uint32_t)F; o.score = M; o.ties = (uint32_t)ties; o.rec = -1;
      o.ds_norm = (int32_t)(p.ds_on ? dsn : 0); o.rs_norm = (int32_t)(p.rs_on ? rsn : 0); o.pref_node = pref;
      o.err = err;
      *out = o;
    }
  }
}

constexpr int DEV_WORDS = (int)(sizeof(DevNode) / 8);
static_assert(sizeof(DevNode) % 8 == 0, "DevNode words");
__global__ __launch_bounds__(256) void scatter_devnodes_kernel(DevNode* dev, const uint32_t* __restrict__ idx,
                                                               const DevNode* __restrict__ img, uint32_t n) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n * DEV_WORDS) return;
  const uint32_t j = t / DEV_WORDS, w = t % DEV_WORDS;
  reinterpret_cast<int64_t*>(dev + idx[j])[w] = reinterpret_cast<const int64_t*>(img + j)[w];
}

}  // namespace

hipError_t launch_scatter_devnodes(DevNode* dev, const uint32_t* idx, const DevNode* img, uint32_t n, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(scatter_devnodes_kernel, dim3((n * DEV_WORDS + 255) / 256), dim3(256), 0, st, dev, idx, img, n);
  return hipGetLastError();
}

hipError_t launch_ext_nodes(const DevNode* dev, const int16_t* S, uint32_t n0, uint32_t n1, const ExtPod* pod,
                            int32_t* tot, int16_t* ds, int16_t* rs, int32_t* scratch, hipStream_t st) {
  const uint32_t len = n1 - n0;
  hipLaunchKernelGGL(ext_nodes_kernel, dim3(len ? (len + 255) / 256 : 1), dim3(256), 0, st, dev, S, n0, n1, pod, tot,
                     ds, rs, scratch + len);
  return hipGetLastError();
}

hipError_t launch_ext_matched(const MirrorView& m, const PodVec* pods, const Profile& pf, int prod_cols,
                              const DevNode* dev, const ExtPod* pod, const ExtRec* recs, const ExtRes* res, int nrec, int32_t* tot,
                              int16_t* ds, int16_t* rs, int32_t* nominated, uint8_t* aff, uint32_t n0, int32_t* scratch,
                              uint32_t len, hipStream_t st) {
  // scratch: T[len] | acc[ACC_WORDS] | bcnt[blocks]; the accumulators were reset by ext_nodes_kernel
  int32_t* acc = scratch + len;
  hipLaunchKernelGGL(ext_matched_kernel, dim3(1), dim3(SEL_BLOCK), 0, st, m, pods, pf, prod_cols, dev, pod, recs, res, nrec,
                     tot, ds, rs, nominated, aff, n0, acc);
  return hipGetLastError();
}

hipError_t launch_ext_select(const int32_t* tot, const int16_t* ds, const int16_t* rs, const ExtRec* recs, uint32_t n0,
                             uint32_t n1, const ExtPod* pod, uint64_t seed, int32_t* scratch, ExtOut* out,
                             hipStream_t st) {
  const uint32_t len = n1 - n0;
  const uint32_t blocks = len ? (len + SEL_SPAN - 1) / SEL_SPAN : 1;
  int32_t* T = scratch;
  int32_t* acc = scratch + len;
  int32_t* bcnt = acc + ACC_WORDS;
  hipLaunchKernelGGL(ext_acc_kernel, dim3(blocks), dim3(SEL_BLOCK), 0, st, tot, ds, rs, recs, n0, len, pod, acc);
  hipLaunchKernelGGL(ext_total_kernel, dim3(blocks), dim3(SEL_BLOCK), 0, st, tot, ds, rs, recs, n0, len, pod, T, acc);
  hipLaunchKernelGGL(ext_ties_kernel, dim3(blocks), dim3(SEL_BLOCK), 0, st, T, ds, rs, n0, len, pod, seed, acc, bcnt,
                     out);
  return hipGetLastError();
}

hipError_t launch_ext_numa(const MirrorView& m, const PodVec* pods, const Profile& pf, int prod_cols, const DevNode* dev,
                           const ExtPod* pod, const uint32_t* idx, uint32_t nidx, uint32_t n0, int32_t* tot, int16_t* ds,
                           uint8_t* aff, int32_t* scratch, uint32_t len, hipStream_t st) {
  if (!nidx) return hipSuccess;
  hipLaunchKernelGGL(ext_numa_kernel, dim3((nidx + 255) / 256), dim3(256), 0, st, m, pods, pf, prod_cols, dev, pod, idx,
                     nidx, n0, tot, ds, aff, scratch + len);
  return hipGetLastError();
}

hipError_t launch_ext_finish(const MirrorView& m, const PodVec* pods, const Profile& pf, int prod_cols,
                             const uint8_t* aff, uint32_t n0, int numa, const ExtOut* out, const int32_t* nom, int nrec,
                             ExtOut* host_out, int32_t* host_nom, hipStream_t st) {
  hipLaunchKernelGGL(ext_finish_kernel, dim3(1), dim3(64), 0, st, m, pods, pf, prod_cols, aff, n0, numa, out, nom, nrec,
                     host_out, host_nom);
  return hipGetLastError();
}

size_t ext_select_scratch_words(uint32_t len) { return len + ACC_WORDS + (len + SEL_BLOCK - 1) / SEL_BLOCK + 64; }

}  // namespace gs

// gs_cpuset_dev.h — cpuset selection of NodeNUMAResource Reserve (resourceManager.allocateCPUSet,
// nodenumaresource/resource_manager.go:273-360 -> takeCPUs, cpu_accumulator.go:87-232, and the
// cpuAccumulator list builders :234-822) over core bit planes, so that the commit kernel can Reserve a
// cpuset pod on the device and keep the batch going. The same code is compiled for the host, where the
// library self-test (gsx_cpuset_selftest) compares it with the host restatement (gs_numa_host.cpp take_cpus).
//
// Scope (TopoDev.ok, "compact" topologies): <= 64 cores of <= 4 CPUs, <= 8 NUMA nodes and sockets, every
// core and every NUMA node inside one socket; the node's maxRefCount <= 1 (no RefCount ordering). Nodes
// outside it keep the host path (the commit kernel ends the batch after such a pod).
//
// Representation: core rank k = position of the core id in ascending order (the reference's core-id
// tiebreaks), NUMA node / socket index = position of the id in ascending order, CPU position j = rank of
// the CPU id inside its core. A set of CPUs is 4 planes of 64-bit core masks: plane j, bit k = CPU (k, j).
// Lists the reference orders by CPU id are materialised as 256-bit CPU masks (cpu_core / cpu_pos map back).
#pragma once
#include <stdint.h>

#include "../../include/gpuscore.h"

#if defined(__HIP__)
#define GS_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define GS_HD inline
#endif

namespace gs {

constexpr int TD_CORES = 64, TD_NODES = 8, TD_SOCKETS = 8, TD_POS = 4;

struct TopoDev {
  int32_t ok;                       // the device path applies to this topology
  int32_t num_cpus, ncores, cpc, cpn, cps, nnodes, nsockets;
  uint64_t node_cores[TD_NODES];    // cores of NUMA node index n
  uint64_t sock_cores[TD_SOCKETS];  // cores of socket index s
  uint64_t pos_cores[TD_POS];       // cores with a CPU at position j
  uint8_t core_node[TD_CORES];
  uint8_t node_sock[TD_NODES];
  uint8_t pad[8];
  uint8_t core_cpu[TD_CORES][TD_POS];
  uint8_t cpu_core[256];
  uint8_t cpu_pos[256];
};
static_assert(sizeof(TopoDev) % 8 == 0, "TopoDev is staged to LDS as 64-bit words");

// Per-node CPU state the device Reserve reads and updates (HBM columns C_CPU_UN0.. / C_CPU_META).
struct CpuStateDev {
  uint64_t un[TD_POS];   // not available: allocated (RefCount > 0) or reserved
  uint64_t xc;           // cores holding an allocated CPU with PCPULevel exclusivity
  uint64_t zal;          // allocated CPUs per zone slot z (16 bits each)
  uint32_t meta;         // CM_* below
  int32_t topo;          // TopoDev index; -1: cpuset selection stays on the host
};
enum : uint32_t {
  CM_XN_MASK = 0xFFu,    // NUMA node indexes holding a NUMANodeLevel-exclusive allocated CPU
  CM_ZIDX_SHIFT = 8,     // 4 x 4 bits: zone slot z -> NUMA node index (0xF: not in the topology)
  CM_MOST = 1u << 24,    // NUMAAllocateStrategy MostAllocated (GetNUMAAllocateStrategy, util.go:35-41)
};

GS_HD int td_pc(uint64_t x) { return __builtin_popcountll(x); }
GS_HD int td_ctz(uint64_t x) { return __builtin_ctzll(x); }
GS_HD int td_cnt(const uint64_t* P, uint64_t m) {
  return td_pc(P[0] & m) + td_pc(P[1] & m) + td_pc(P[2] & m) + td_pc(P[3] & m);
}
GS_HD uint64_t td_any(const uint64_t* P) { return P[0] | P[1] | P[2] | P[3]; }
GS_HD uint64_t td_all(const TopoDev& t) { return t.ncores >= 64 ? ~0ull : ((1ull << t.ncores) - 1ull); }

// E[v] = cores with exactly v CPUs set in P (v = 0..4), bit-sliced
GS_HD void td_exact(const uint64_t* P, uint64_t* E) {
  const uint64_t s0 = P[0] ^ P[1], c0 = P[0] & P[1], s1 = P[2] ^ P[3], c1 = P[2] & P[3];
  const uint64_t b0 = s0 ^ s1, t1 = s0 & s1;
  const uint64_t b1 = c0 ^ c1 ^ t1, b2 = (c0 & c1) | (c0 & t1) | (c1 & t1);
  E[0] = ~b0 & ~b1 & ~b2;
  E[1] = b0 & ~b1 & ~b2;
  E[2] = ~b0 & b1 & ~b2;
  E[3] = b0 & b1 & ~b2;
  E[4] = ~b0 & ~b1 & b2;
}

// position of the r-th set CPU of core k in P (-1: none)
GS_HD int td_rth(const uint64_t* P, int k, int r) {
  for (int j = 0; j < TD_POS; ++j)
    if ((P[j] >> k) & 1u) {
      if (r == 0) return j;
      --r;
    }
  return -1;
}

// cpuAccumulator (cpu_accumulator.go:234-330) with maxRefCount <= 1
struct DAcc {
  const TopoDev& t;
  uint64_t A[TD_POS];   // allocatableCPUs
  uint64_t R[TD_POS];   // result
  uint64_t xc;          // exclusiveInCores
  uint32_t xn;          // exclusiveInNUMANodes (node indexes)
  int needed, nalloc, ep;
  bool most, exclusive;

  GS_HD DAcc(const TopoDev& tt, const uint64_t* avail, uint64_t xc0, uint32_t xn0, int n, int e, bool m)
      : t(tt), xc(xc0), xn(xn0), needed(n), ep(e), most(m) {
    for (int j = 0; j < TD_POS; ++j) { A[j] = avail[j]; R[j] = 0; }
    nalloc = td_cnt(A, ~0ull);
    exclusive = e == GS_CPU_EXCLUSIVE_PCPU_LEVEL || e == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL;
  }
  GS_HD bool sless(int a, int b) const { return most ? a < b : a > b; }
  GS_HD int dir(int x) const { return most ? x : 511 - x; }   // ascending key of the sless order
  GS_HD bool satisfied() const { return needed < 1; }
  GS_HD uint64_t nodes_cores(uint32_t nodes) const {
    uint64_t m = 0;
    for (; nodes; nodes &= nodes - 1) m |= t.node_cores[td_ctz(nodes)];
    return m;
  }
  // filterExclusive predicates: isCPUExclusivePCPULevel / isCPUExclusiveNUMANodeLevel (:318-330)
  GS_HD uint64_t keep_xp(bool fe) const { return (fe && ep == GS_CPU_EXCLUSIVE_PCPU_LEVEL) ? ~xc : ~0ull; }
  GS_HD uint64_t keep_xn(bool fe) const {
    return (fe && ep == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL) ? ~nodes_cores(xn) : ~0ull;
  }
  GS_HD void take(int k, int j) {   // take (:290-304)
    const uint64_t b = 1ull << k;
    R[j] |= b;
    if (A[j] & b) { A[j] &= ~b; --nalloc; }
    --needed;
    if (exclusive) {
      if (ep == GS_CPU_EXCLUSIVE_PCPU_LEVEL) xc |= b;
      else xn |= 1u << t.core_node[k];
    }
  }
  // the first `n` allocatable CPUs of core k in CPU order
  GS_HD void take_core(int k, int n) {
    for (int j = 0; j < TD_POS && n > 0; ++j)
      if ((A[j] >> k) & 1u) { take(k, j); --n; }
  }
  // head(list, needed) of a full-core list (cores ascending, CPUs ascending)
  GS_HD void take_head_cores(uint64_t q) {
    for (; q && needed > 0; q &= q - 1) take_core(td_ctz(q), needed < t.cpc ? needed : t.cpc);
  }
  // Takes up to `needed` CPUs, in CPU-id order, out of the pass-r CPUs (the r-th CPU of each core) of the
  // snapshot S; r < 0: all CPUs of S.
  GS_HD void take_cpu_order(const uint64_t* S, int r) {
    uint64_t W[4] = {0, 0, 0, 0};
    for (uint64_t b = td_any(S); b; b &= b - 1) {
      const int k = td_ctz(b);
      if (r < 0) {
        for (int j = 0; j < TD_POS; ++j)
          if ((S[j] >> k) & 1u) {
            const int c = t.core_cpu[k][j];
            W[c >> 6] |= 1ull << (c & 63);
          }
      } else {
        const int j = td_rth(S, k, r);
        if (j < 0) continue;
        const int c = t.core_cpu[k][j];
        W[c >> 6] |= 1ull << (c & 63);
      }
    }
    for (int w = 0; w < 4; ++w)
      for (; W[w] && needed > 0; W[w] &= W[w] - 1) {
        const int c = w * 64 + td_ctz(W[w]);
        take(t.cpu_core[c], t.cpu_pos[c]);
      }
  }
  // head(spreadCPUs(list), needed) for a list in CPU-id order: the CPUs of cores `m` in A; `first_only`:
  // the list went through extractCPU (one CPU per core), L = its length
  GS_HD void take_spread_cpu_list(uint64_t m, bool first_only, int L) {
    uint64_t S[TD_POS];
    for (int j = 0; j < TD_POS; ++j) S[j] = A[j] & m;
    if (!first_only && L <= t.cpc) { take_cpu_order(S, -1); return; }   // spreadCPUs keeps short lists as is
    const int passes = first_only ? 1 : TD_POS;
    for (int r = 0; r < passes && needed > 0; ++r) take_cpu_order(S, r);
  }
  GS_HD uint64_t full_cores(uint64_t keep) const {
    uint64_t K[TD_POS], E[5];
    for (int j = 0; j < TD_POS; ++j) K[j] = A[j] & keep;
    td_exact(K, E);
    return E[t.cpc] & td_any(K);
  }
  // freeCoresInNode(true, fe) (:370-461): the first NUMA node list with >= needed CPUs (-1: none)
  GS_HD int pick_full_node(bool fe, uint64_t* cores) const {
    const uint64_t keep = td_all(t) & keep_xn(fe);
    const uint64_t full = full_cores(keep);
    int best = -1, bsz = 0, bsf = 0;
    for (int n = 0; n < t.nnodes; ++n) {
      const uint64_t q = full & t.node_cores[n];
      if (!q) continue;
      const int sz = t.cpc * td_pc(q);
      if (sz < needed) continue;
      const int sf = td_cnt(A, keep & t.sock_cores[t.node_sock[n]]);
      if (best < 0 || sless(sz, bsz) || (sz == bsz && sless(sf, bsf))) { best = n; bsz = sz; bsf = sf; *cores = q; }
    }
    return best;
  }
  // freeCoresInSocket(true) (:463-527): the first socket list with >= needed CPUs
  GS_HD int pick_full_socket(uint64_t* cores) const {
    const uint64_t full = full_cores(~0ull);
    int best = -1, bsz = 0;
    for (int s = 0; s < t.nsockets; ++s) {
      const uint64_t q = full & t.sock_cores[s];
      if (!q) continue;
      const int sz = t.cpc * td_pc(q);
      if (sz < needed) continue;
      if (best < 0 || sless(sz, bsz)) { best = s; bsz = sz; *cores = q; }
    }
    return best;
  }
  // freeCPUsInNode(fe) (:529-605): the first NUMA node list with >= needed CPUs
  GS_HD int pick_cpus_node(bool fe, uint64_t* cores, int* L) const {
    const uint64_t keep = td_all(t) & keep_xp(fe) & keep_xn(fe);
    int best = -1, bnf = 0, bsf = 0;
    for (int n = 0; n < t.nnodes; ++n) {
      const uint64_t m = keep & t.node_cores[n];
      const int nf = td_cnt(A, m);
      if (nf == 0) continue;
      const int len = fe ? td_pc(td_any(A) & m) : nf;
      if (len < needed) continue;
      const int sf = td_cnt(A, keep & t.sock_cores[t.node_sock[n]]);
      if (best < 0 || sless(nf, bnf) || (nf == bnf && sless(sf, bsf))) {
        best = n; bnf = nf; bsf = sf; *cores = m; *L = len;
      }
    }
    return best;
  }
  // freeCPUsInSocket(fe) (:607-656)
  GS_HD int pick_cpus_socket(bool fe, uint64_t* cores, int* L) const {
    const uint64_t keep = td_all(t) & keep_xp(fe);
    int best = -1, bl = 0;
    for (int s = 0; s < t.nsockets; ++s) {
      const uint64_t m = keep & t.sock_cores[s];
      const int nf = td_cnt(A, m);
      if (nf == 0) continue;
      const int len = fe ? td_pc(td_any(A) & m) : nf;
      if (len < needed) continue;
      if (best < 0 || sless(len, bl)) { best = s; bl = len; *cores = m; *L = len; }
    }
    return best;
  }
  // head(spreadCPUs(freeCPUs(fe)), needed) (:658-774): cores ordered by (CPUs of the result in the socket
  // desc, socket free, node free, core size asc, socket id, core id), CPUs of a core ascending
  GS_HD void take_free_cpus(bool fe) {
    const uint64_t keep = td_all(t) & keep_xp(fe) & keep_xn(fe);
    uint64_t S[TD_POS], E[5];
    for (int j = 0; j < TD_POS; ++j) S[j] = A[j] & keep;
    const uint64_t cores = td_any(S);
    if (!cores) return;
    td_exact(S, E);
    const int L = td_cnt(S, ~0ull);
    // NUMA nodes by group key (colo desc, socket free, node free), ascending; equal keys merge
    uint32_t key[TD_NODES];
    int ord[TD_NODES], nn = 0;
    for (int n = 0; n < t.nnodes; ++n) {
      if (!(cores & t.node_cores[n])) continue;
      const uint64_t sm = t.sock_cores[t.node_sock[n]];
      const int colo = td_cnt(R, sm), sf = td_cnt(S, sm), nf = td_cnt(S, t.node_cores[n]);
      key[n] = ((uint32_t)(511 - colo) << 18) | ((uint32_t)dir(sf) << 9) | (uint32_t)dir(nf);
      int i = nn++;
      while (i > 0 && key[ord[i - 1]] > key[n]) { ord[i] = ord[i - 1]; --i; }
      ord[i] = n;
    }
    const bool as_is = L <= t.cpc;   // spreadCPUs keeps short lists as is
    const int passes = as_is ? 1 : TD_POS;
    for (int r = 0; r < passes; ++r) {
      for (int g = 0; g < nn;) {
        uint64_t M = 0;
        int h = g;
        for (; h < nn && key[ord[h]] == key[ord[g]]; ++h) M |= cores & t.node_cores[ord[h]];
        g = h;
        for (int v = 1; v <= TD_POS; ++v) {
          if (!as_is && v <= r) continue;
          const uint64_t Mv = M & E[v];
          if (!Mv) continue;
          for (int s = 0; s < t.nsockets; ++s)
            for (uint64_t q = Mv & t.sock_cores[s]; q; q &= q - 1) {
              const int k = td_ctz(q);
              if (as_is) {
                for (int j = 0; j < TD_POS && needed > 0; ++j)
                  if ((S[j] >> k) & 1u) take(k, j);
              } else {
                take(k, td_rth(S, k, r));
              }
              if (needed < 1) return;
            }
        }
      }
    }
  }
};

// Go 1.18 sort.Slice on <= 12 elements: gap-6 pass + insertion sort (as gs_numa_host.cpp go_sort_small)
GS_HD void td_go_sort(int* id, int* sz, int n, bool desc) {
  for (int i = 6; i < n; ++i)
    if (desc ? sz[i] > sz[i - 6] : sz[i] < sz[i - 6]) {
      int x = id[i]; id[i] = id[i - 6]; id[i - 6] = x;
      x = sz[i]; sz[i] = sz[i - 6]; sz[i - 6] = x;
    }
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && (desc ? sz[j] > sz[j - 1] : sz[j] < sz[j - 1]); --j) {
      int x = id[j]; id[j] = id[j - 1]; id[j - 1] = x;
      x = sz[j]; sz[j] = sz[j - 1]; sz[j - 1] = x;
    }
}

// takeCPUs (cpu_accumulator.go:87-232); avail = planes of the CPUs it may take. false: the reference errors.
GS_HD bool td_take_cpus(const TopoDev& t, const uint64_t* avail, uint64_t xc, uint32_t xn, int needed,
                               int bind, int ep, bool most, uint64_t* out) {
  DAcc a(t, avail, xc, xn, needed, ep, most);
  for (int j = 0; j < TD_POS; ++j) out[j] = 0;
  if (a.satisfied()) return true;
  if (a.needed > a.nalloc) return false;
  const bool full = bind == GS_CPU_BIND_FULL_PCPUS;
  bool ok = false;
  do {
    uint64_t m = 0;
    int L = 0;
    if (full || t.cpc == 1) {
      if (a.needed <= t.cpn && (a.pick_full_node(true, &m) >= 0 || a.pick_full_node(false, &m) >= 0)) {
        a.take_head_cores(m);
        ok = true;
        break;
      }
      if (a.needed <= t.cps && a.pick_full_socket(&m) >= 0) {
        a.take_head_cores(m);
        ok = true;
        break;
      }
      // freeCoresInSocket(true) in (size, id) order, then sort.Slice by size desc (:141-155)
      const uint64_t fc = a.full_cores(~0ull);
      int id[TD_SOCKETS], sz[TD_SOCKETS], ns = 0;
      for (int s = 0; s < t.nsockets; ++s) {
        const uint64_t q = fc & t.sock_cores[s];
        if (!q) continue;
        const int z = t.cpc * td_pc(q);
        int i = ns++;
        while (i > 0 && a.sless(z, sz[i - 1])) { id[i] = id[i - 1]; sz[i] = sz[i - 1]; --i; }
        id[i] = s;
        sz[i] = z;
      }
      td_go_sort(id, sz, ns, true);
      int uid[TD_SOCKETS], usz[TD_SOCKETS], nu = 0;
      for (int i = 0; i < ns && !ok; ++i) {
        if (a.needed < sz[i]) { uid[nu] = id[i]; usz[nu] = sz[i]; ++nu; continue; }
        for (uint64_t b = fc & t.sock_cores[id[i]]; b; b &= b - 1) a.take_core(td_ctz(b), TD_POS);
        ok = a.satisfied();
      }
      if (ok) break;
      if (a.needed >= t.cpc) {   // (:157-176)
        td_go_sort(uid, usz, nu, false);
        for (int i = 0; i < nu && !ok; ++i)
          for (uint64_t b = fc & t.sock_cores[uid[i]]; b; b &= b - 1) {
            a.take_core(td_ctz(b), TD_POS);
            if (a.satisfied()) { ok = true; break; }
            if (a.needed < t.cpc) break;
          }
        if (ok) break;
      }
    }
    if (!full) {   // (:184-215)
      if (a.needed <= t.cpn) {
        if (a.pick_cpus_node(true, &m, &L) >= 0) { a.take_spread_cpu_list(m, true, L); ok = true; break; }
        if (a.pick_cpus_node(false, &m, &L) >= 0) { a.take_spread_cpu_list(m, false, L); ok = true; break; }
      }
      if (a.needed <= t.cps) {
        if (a.pick_cpus_socket(true, &m, &L) >= 0) { a.take_spread_cpu_list(m, true, L); ok = true; break; }
        if (a.pick_cpus_socket(false, &m, &L) >= 0) { a.take_spread_cpu_list(m, false, L); ok = true; break; }
      }
    }
    a.take_free_cpus(true);   // (:217-229)
    if (a.satisfied()) { ok = true; break; }
    a.take_free_cpus(false);
    ok = a.satisfied();
  } while (false);
  if (!ok) return false;
  for (int j = 0; j < TD_POS; ++j) out[j] = a.R[j];
  return true;
}

// available CPUs (getAvailableCPUs, node_allocation.go:142-162, maxRefCount <= 1) as planes
GS_HD void td_available(const TopoDev& t, const CpuStateDev& cs, uint64_t* P) {
  for (int j = 0; j < TD_POS; ++j) P[j] = t.pos_cores[j] & ~cs.un[j];
}
GS_HD int td_zone_node(const CpuStateDev& cs, int z) { return (int)((cs.meta >> (CM_ZIDX_SHIFT + 4 * z)) & 15u); }

// allocateCPUSet (resource_manager.go:273-360) given the NUMA split Allocate produced (PlacementDev zkeys /
// zcpu). false: the reference errors (cannot follow a feasible Filter; the host fails loudly).
GS_HD bool td_allocate_cpuset(const TopoDev& t, const CpuStateDev& cs, int num_cpus, int bind, bool required,
                                     int ep, uint32_t zkeys, const int64_t* zcpu, uint64_t* out) {
  uint64_t P[TD_POS];
  td_available(t, cs, P);
  const bool most = cs.meta & CM_MOST;
  const uint64_t xc = cs.xc;
  const uint32_t xn = cs.meta & CM_XN_MASK;
  if (required) {   // filterCPUsByRequiredCPUBindPolicy (:534-566)
    if (bind == GS_CPU_BIND_FULL_PCPUS) {
      uint64_t E[5];
      td_exact(P, E);
      const uint64_t f = E[t.cpc] & td_any(P);
      for (int j = 0; j < TD_POS; ++j) P[j] &= f;
    } else if (bind == GS_CPU_BIND_SPREAD_BY_PCPUS) {
      uint64_t seen = 0;
      for (int j = 0; j < TD_POS; ++j) { P[j] &= ~seen; seen |= P[j]; }
    }
  }
  for (int j = 0; j < TD_POS; ++j) out[j] = 0;
  if (td_cnt(P, ~0ull) < num_cpus) return false;
  int needed = num_cpus;
  uint64_t got[TD_POS];
  if (zkeys) {
    for (int z = 0; z < 4; ++z) {
      if (!((zkeys >> z) & 1u) && !((zkeys >> (4 + z)) & 1u)) continue;
      const int n = td_zone_node(cs, z);
      const uint64_t m = n < t.nnodes ? t.node_cores[n] : 0;
      uint64_t in[TD_POS];
      for (int j = 0; j < TD_POS; ++j) in[j] = P[j] & m;
      int num = td_cnt(in, ~0ull);
      const int want = ((zkeys >> z) & 1u) ? (int)(zcpu[z] / 1000) : 0;
      if (want < num) num = want;
      if (num <= 0) continue;   // takePreferredCPUs with nothing needed
      if (!td_take_cpus(t, in, xc, xn, num, bind, ep, most, got)) return false;
      for (int j = 0; j < TD_POS; ++j) out[j] |= got[j];
    }
    needed -= td_cnt(out, ~0ull);
    if (needed != 0) return false;
  }
  if (needed > 0) {
    uint64_t rest[TD_POS];
    for (int j = 0; j < TD_POS; ++j) rest[j] = P[j] & ~out[j];
    if (!td_take_cpus(t, rest, xc, xn, needed, bind, ep, most, got)) return false;
    for (int j = 0; j < TD_POS; ++j) out[j] |= got[j];
  }
  if (required) {   // satisfiedRequiredCPUBindPolicy (:568-589)
    const int nc = td_pc(td_any(out)), ncpus = td_cnt(out, ~0ull);
    if (bind == GS_CPU_BIND_FULL_PCPUS && nc * t.cpc != ncpus) return false;
    if (bind == GS_CPU_BIND_SPREAD_BY_PCPUS && nc != ncpus) return false;
  }
  return true;
}

// available-CPU counts of the cores `m` (raw | full-core CPUs << 9 | cores with a free CPU << 18), packed
// as gs_numa_host.cpp count_available
GS_HD int32_t td_counts(const TopoDev& t, const CpuStateDev& cs, uint64_t m) {
  uint64_t P[TD_POS], E[5];
  td_available(t, cs, P);
  for (int j = 0; j < TD_POS; ++j) P[j] &= m;
  td_exact(P, E);
  const int raw = td_cnt(P, ~0ull);
  const int full = t.cpc * td_pc(E[t.cpc] & td_any(P));
  const int spread = td_pc(td_any(P));
  return (int32_t)(raw | (full << 9) | (spread << 18));
}

// the cpuset as a 256-bit CPU mask
GS_HD void td_to_cpus(const TopoDev& t, const uint64_t* R, uint64_t* w) {
  w[0] = w[1] = w[2] = w[3] = 0;
  for (int j = 0; j < TD_POS; ++j)
    for (uint64_t b = R[j]; b; b &= b - 1) {
      const int c = t.core_cpu[td_ctz(b)][j];
      w[c >> 6] |= 1ull << (c & 63);
    }
}

}  // namespace gs

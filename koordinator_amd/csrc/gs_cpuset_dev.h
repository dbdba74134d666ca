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

// Wave-uniform reads of the topology / CPU state: on the device these functions run for one Reserve at a time (one
// active lane or identical operands in every lane), so a value read from LDS is moved to a scalar register and the
// selection below runs on the scalar unit (64-bit masks natively) instead of one VALU lane.
GS_HD int32_t TU32(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_readfirstlane(x);
#else
  return x;
#endif
}
GS_HD uint32_t TUU(uint32_t x) { return (uint32_t)TU32((int32_t)x); }
GS_HD uint64_t TU64(uint64_t x) { return ((uint64_t)TUU((uint32_t)(x >> 32)) << 32) | TUU((uint32_t)x); }

GS_HD int td_pc(uint64_t x) { return __builtin_popcountll(x); }
GS_HD int td_ctz(uint64_t x) { return __builtin_ctzll(x); }
GS_HD int td_cnt(const uint64_t* P, uint64_t m) {
  return td_pc(P[0] & m) + td_pc(P[1] & m) + td_pc(P[2] & m) + td_pc(P[3] & m);
}
GS_HD uint64_t td_any(const uint64_t* P) { return P[0] | P[1] | P[2] | P[3]; }
GS_HD uint64_t td_all(const TopoDev& t) { return TU32(t.ncores) >= 64 ? ~0ull : ((1ull << TU32(t.ncores)) - 1ull); }

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

// cores with exactly v CPUs set in P, v a run-time value (no indexed register array: on the device a dynamically
// indexed local array lives in scratch memory)
GS_HD uint64_t td_exactly(const uint64_t* P, int v) {
  uint64_t E[5];
  td_exact(P, E);
  return v == 0 ? E[0] : v == 1 ? E[1] : v == 2 ? E[2] : v == 3 ? E[3] : v == 4 ? E[4] : 0ull;
}
// 8 run-time-indexed 32-bit entries in four named 64-bit registers (a local array indexed at run time would
// live in scratch memory on the device)
struct TdPack8 {
  uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  GS_HD uint32_t get(int i) const {
    const int h = i >> 1;
    const uint64_t w = h == 0 ? w0 : h == 1 ? w1 : h == 2 ? w2 : w3;
    return (uint32_t)(w >> (32 * (i & 1)));
  }
  GS_HD void set(int i, uint32_t v) {
    const int h = i >> 1, sh = 32 * (i & 1);
    const uint64_t keep = ~(0xFFFFFFFFull << sh), put = (uint64_t)v << sh;
    w0 = h == 0 ? (w0 & keep) | put : w0;
    w1 = h == 1 ? (w1 & keep) | put : w1;
    w2 = h == 2 ? (w2 & keep) | put : w2;
    w3 = h == 3 ? (w3 & keep) | put : w3;
  }
};
// a 256-bit CPU mask in four named registers
struct TdMask256 {
  uint64_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  GS_HD void set_bit(int c) {
    const uint64_t b = 1ull << (c & 63);
    const int h = c >> 6;
    w0 |= h == 0 ? b : 0ull;
    w1 |= h == 1 ? b : 0ull;
    w2 |= h == 2 ? b : 0ull;
    w3 |= h == 3 ? b : 0ull;
  }
};

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
    for (; nodes; nodes &= nodes - 1) m |= TU64(t.node_cores[td_ctz(nodes)]);
    return m;
  }
  // filterExclusive predicates: isCPUExclusivePCPULevel / isCPUExclusiveNUMANodeLevel (:318-330)
  GS_HD uint64_t keep_xp(bool fe) const { return (fe && ep == GS_CPU_EXCLUSIVE_PCPU_LEVEL) ? ~xc : ~0ull; }
  GS_HD uint64_t keep_xn(bool fe) const {
    return (fe && ep == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL) ? ~nodes_cores(xn) : ~0ull;
  }
  GS_HD void take(int k, int j) {   // take (:290-304)
    const uint64_t b = 1ull << k;
#pragma unroll
    for (int jj = 0; jj < TD_POS; ++jj) {
      if (jj != j) continue;
      R[jj] |= b;
      if (A[jj] & b) { A[jj] &= ~b; --nalloc; }
    }
    --needed;
    if (exclusive) {
      if (ep == GS_CPU_EXCLUSIVE_PCPU_LEVEL) xc |= b;
      else xn |= 1u << TU32(t.core_node[k]);
    }
  }
  // the first `n` allocatable CPUs of core k in CPU order
  GS_HD void take_core(int k, int n) {
#pragma unroll
    for (int j = 0; j < TD_POS; ++j)
      if (n > 0 && ((A[j] >> k) & 1u)) { take(k, j); --n; }
  }
  // head(list, needed) of a full-core list (cores ascending, CPUs ascending)
  GS_HD void take_head_cores(uint64_t q) {
    for (; q && needed > 0; q &= q - 1) take_core(td_ctz(q), needed < TU32(t.cpc) ? needed : TU32(t.cpc));
  }
  // Takes up to `needed` CPUs, in CPU-id order, out of the pass-r CPUs (the r-th CPU of each core) of the
  // snapshot S; r < 0: all CPUs of S.
  GS_HD void take_cpu_order(const uint64_t* S, int r) {
    TdMask256 W;
    for (uint64_t b = td_any(S); b; b &= b - 1) {
      const int k = td_ctz(b);
      if (r < 0) {
#pragma unroll
        for (int j = 0; j < TD_POS; ++j)
          if ((S[j] >> k) & 1u) {
            W.set_bit(TU32(t.core_cpu[k][j]));
          }
      } else {
        const int j = td_rth(S, k, r);
        if (j < 0) continue;
        W.set_bit(TU32(t.core_cpu[k][j]));
      }
    }
#pragma unroll
    for (int w = 0; w < 4; ++w)
      for (uint64_t x = w == 0 ? W.w0 : w == 1 ? W.w1 : w == 2 ? W.w2 : W.w3; x && needed > 0; x &= x - 1) {
        const int c = w * 64 + td_ctz(x);
        take(TU32(t.cpu_core[c]), TU32(t.cpu_pos[c]));
      }
  }
  // head(spreadCPUs(list), needed) for a list in CPU-id order: the CPUs of cores `m` in A; `first_only`:
  // the list went through extractCPU (one CPU per core), L = its length
  GS_HD void take_spread_cpu_list(uint64_t m, bool first_only, int L) {
    uint64_t S[TD_POS];
    for (int j = 0; j < TD_POS; ++j) S[j] = A[j] & m;
    if (!first_only && L <= TU32(t.cpc)) { take_cpu_order(S, -1); return; }   // spreadCPUs keeps short lists as is
    const int passes = first_only ? 1 : TD_POS;
    for (int r = 0; r < passes && needed > 0; ++r) take_cpu_order(S, r);
  }
  GS_HD uint64_t full_cores(uint64_t keep) const {
    uint64_t K[TD_POS];
    for (int j = 0; j < TD_POS; ++j) K[j] = A[j] & keep;
    return td_exactly(K, TU32(t.cpc)) & td_any(K);
  }
  // freeCoresInNode(true, fe) (:370-461): the first NUMA node list with >= needed CPUs (-1: none)
  GS_HD int pick_full_node(bool fe, uint64_t* cores) const {
    const uint64_t keep = td_all(t) & keep_xn(fe);
    const uint64_t full = full_cores(keep);
    int best = -1, bsz = 0, bsf = 0;
    for (int n = 0; n < TU32(t.nnodes); ++n) {
      const uint64_t q = full & TU64(t.node_cores[n]);
      if (!q) continue;
      const int sz = TU32(t.cpc) * td_pc(q);
      if (sz < needed) continue;
      const int sf = td_cnt(A, keep & TU64(t.sock_cores[TU32(t.node_sock[n])]));
      if (best < 0 || sless(sz, bsz) || (sz == bsz && sless(sf, bsf))) { best = n; bsz = sz; bsf = sf; *cores = q; }
    }
    return best;
  }
  // freeCoresInSocket(true) (:463-527): the first socket list with >= needed CPUs
  GS_HD int pick_full_socket(uint64_t* cores) const {
    const uint64_t full = full_cores(~0ull);
    int best = -1, bsz = 0;
    for (int s = 0; s < TU32(t.nsockets); ++s) {
      const uint64_t q = full & TU64(t.sock_cores[s]);
      if (!q) continue;
      const int sz = TU32(t.cpc) * td_pc(q);
      if (sz < needed) continue;
      if (best < 0 || sless(sz, bsz)) { best = s; bsz = sz; *cores = q; }
    }
    return best;
  }
  // freeCPUsInNode(fe) (:529-605): the first NUMA node list with >= needed CPUs
  GS_HD int pick_cpus_node(bool fe, uint64_t* cores, int* L) const {
    const uint64_t keep = td_all(t) & keep_xp(fe) & keep_xn(fe);
    int best = -1, bnf = 0, bsf = 0;
    for (int n = 0; n < TU32(t.nnodes); ++n) {
      const uint64_t m = keep & TU64(t.node_cores[n]);
      const int nf = td_cnt(A, m);
      if (nf == 0) continue;
      const int len = fe ? td_pc(td_any(A) & m) : nf;
      if (len < needed) continue;
      const int sf = td_cnt(A, keep & TU64(t.sock_cores[TU32(t.node_sock[n])]));
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
    for (int s = 0; s < TU32(t.nsockets); ++s) {
      const uint64_t m = keep & TU64(t.sock_cores[s]);
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
    // entry i = (key << 3 | node) of the i-th node in key order (stable)
    TdPack8 ok;
    int nn = 0;
    for (int n = 0; n < TU32(t.nnodes); ++n) {
      if (!(cores & TU64(t.node_cores[n]))) continue;
      const uint64_t sm = TU64(t.sock_cores[TU32(t.node_sock[n])]);
      const int colo = td_cnt(R, sm), sf = td_cnt(S, sm), nf = td_cnt(S, TU64(t.node_cores[n]));
      const uint32_t kn = ((uint32_t)(511 - colo) << 18) | ((uint32_t)dir(sf) << 9) | (uint32_t)dir(nf);
      int i = nn++;   // insertion after the last key <= kn (stable)
      while (i > 0 && (ok.get(i - 1) >> 3) > kn) { ok.set(i, ok.get(i - 1)); --i; }
      ok.set(i, kn << 3 | (uint32_t)n);
    }
    const bool as_is = L <= TU32(t.cpc);   // spreadCPUs keeps short lists as is
    const int passes = as_is ? 1 : TD_POS;
    for (int r = 0; r < passes; ++r) {
      for (int g = 0; g < nn;) {
        uint64_t M = 0;
        int h = g;
        const uint32_t kg = ok.get(g) >> 3;
        for (; h < nn && (ok.get(h) >> 3) == kg; ++h) M |= cores & TU64(t.node_cores[ok.get(h) & 7u]);
        g = h;
#pragma unroll
        for (int v = 1; v <= TD_POS; ++v) {
          if (!as_is && v <= r) continue;
          const uint64_t Mv = M & E[v];
          if (!Mv) continue;
          for (int s = 0; s < TU32(t.nsockets); ++s)
            for (uint64_t q = Mv & TU64(t.sock_cores[s]); q; q &= q - 1) {
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
// entries (size << 3 | socket index)
GS_HD void td_go_sort(TdPack8& e, int n, bool desc) {
  auto less = [&](uint32_t a, uint32_t b) { return desc ? (a >> 3) > (b >> 3) : (a >> 3) < (b >> 3); };
  for (int i = 6; i < n; ++i) {
    const uint32_t a = e.get(i), b = e.get(i - 6);
    if (less(a, b)) { e.set(i, b); e.set(i - 6, a); }
  }
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0; --j) {
      const uint32_t a = e.get(j), b = e.get(j - 1);
      if (!less(a, b)) break;
      e.set(j, b);
      e.set(j - 1, a);
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
    if (full || TU32(t.cpc) == 1) {
      if (a.needed <= TU32(t.cpn) && (a.pick_full_node(true, &m) >= 0 || a.pick_full_node(false, &m) >= 0)) {
        a.take_head_cores(m);
        ok = true;
        break;
      }
      if (a.needed <= TU32(t.cps) && a.pick_full_socket(&m) >= 0) {
        a.take_head_cores(m);
        ok = true;
        break;
      }
      // freeCoresInSocket(true) in (size, id) order, then sort.Slice by size desc (:141-155)
      const uint64_t fc = a.full_cores(~0ull);
      TdPack8 so;   // (size << 3 | socket index)
      int ns = 0;
      for (int s = 0; s < TU32(t.nsockets); ++s) {
        const uint64_t q = fc & TU64(t.sock_cores[s]);
        if (!q) continue;
        const int z = TU32(t.cpc) * td_pc(q);
        int i = ns++;
        while (i > 0 && a.sless(z, (int)(so.get(i - 1) >> 3))) { so.set(i, so.get(i - 1)); --i; }
        so.set(i, (uint32_t)z << 3 | (uint32_t)s);
      }
      td_go_sort(so, ns, true);
      TdPack8 uo;
      int nu = 0;
      for (int i = 0; i < ns && !ok; ++i) {
        const uint32_t ei = so.get(i);
        const int idi = (int)(ei & 7u), szi = (int)(ei >> 3);
        if (a.needed < szi) { uo.set(nu++, ei); continue; }
        for (uint64_t b = fc & TU64(t.sock_cores[idi]); b; b &= b - 1) a.take_core(td_ctz(b), TD_POS);
        ok = a.satisfied();
      }
      if (ok) break;
      if (a.needed >= TU32(t.cpc)) {   // (:157-176)
        td_go_sort(uo, nu, false);
        for (int i = 0; i < nu && !ok; ++i)
          for (uint64_t b = fc & TU64(t.sock_cores[uo.get(i) & 7u]); b; b &= b - 1) {
            a.take_core(td_ctz(b), TD_POS);
            if (a.satisfied()) { ok = true; break; }
            if (a.needed < TU32(t.cpc)) break;
          }
        if (ok) break;
      }
    }
    if (!full) {   // (:184-215)
      if (a.needed <= TU32(t.cpn)) {
        if (a.pick_cpus_node(true, &m, &L) >= 0) { a.take_spread_cpu_list(m, true, L); ok = true; break; }
        if (a.pick_cpus_node(false, &m, &L) >= 0) { a.take_spread_cpu_list(m, false, L); ok = true; break; }
      }
      if (a.needed <= TU32(t.cps)) {
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
  for (int j = 0; j < TD_POS; ++j) P[j] = TU64(t.pos_cores[j]) & ~TU64(cs.un[j]);
}
GS_HD int td_zone_node(const CpuStateDev& cs, int z) { return (int)((TUU(cs.meta) >> (CM_ZIDX_SHIFT + 4 * z)) & 15u); }

// allocateCPUSet (resource_manager.go:273-360) given the NUMA split Allocate produced (PlacementDev zkeys /
// zcpu). false: the reference errors (cannot follow a feasible Filter; the host fails loudly).
GS_HD bool td_allocate_cpuset(const TopoDev& t, const CpuStateDev& cs, int num_cpus, int bind, bool required,
                                     int ep, uint32_t zkeys, const int64_t* zcpu, uint64_t* out) {
  uint64_t P[TD_POS];
  td_available(t, cs, P);
  const bool most = TUU(cs.meta) & CM_MOST;
  const uint64_t xc = TU64(cs.xc);
  const uint32_t xn = TUU(cs.meta) & CM_XN_MASK;
  if (required) {   // filterCPUsByRequiredCPUBindPolicy (:534-566)
    if (bind == GS_CPU_BIND_FULL_PCPUS) {
      const uint64_t f = td_exactly(P, TU32(t.cpc)) & td_any(P);
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
      const uint64_t m = n < TU32(t.nnodes) ? TU64(t.node_cores[n]) : 0;
      uint64_t in[TD_POS];
      for (int j = 0; j < TD_POS; ++j) in[j] = P[j] & m;
      int num = td_cnt(in, ~0ull);
      const int64_t zz = z == 0 ? zcpu[0] : z == 1 ? zcpu[1] : z == 2 ? zcpu[2] : zcpu[3];
      const int want = ((zkeys >> z) & 1u) ? (int)(zz / 1000) : 0;
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
    if (bind == GS_CPU_BIND_FULL_PCPUS && nc * TU32(t.cpc) != ncpus) return false;
    if (bind == GS_CPU_BIND_SPREAD_BY_PCPUS && nc != ncpus) return false;
  }
  return true;
}

// available-CPU counts of the cores `m` (raw | full-core CPUs << 9 | cores with a free CPU << 18), packed
// as gs_numa_host.cpp count_available
GS_HD int32_t td_counts(const TopoDev& t, const CpuStateDev& cs, uint64_t m) {
  uint64_t P[TD_POS];
  td_available(t, cs, P);
  for (int j = 0; j < TD_POS; ++j) P[j] &= m;
  const int raw = td_cnt(P, ~0ull);
  const int full = TU32(t.cpc) * td_pc(td_exactly(P, TU32(t.cpc)) & td_any(P));
  const int spread = td_pc(td_any(P));
  return (int32_t)(raw | (full << 9) | (spread << 18));
}

// the cpuset as a 256-bit CPU mask
GS_HD void td_to_cpus(const TopoDev& t, const uint64_t* R, uint64_t* w) {
  TdMask256 W;
#pragma unroll
  for (int j = 0; j < TD_POS; ++j)
    for (uint64_t b = R[j]; b; b &= b - 1) W.set_bit(TU32(t.core_cpu[td_ctz(b)][j]));
  w[0] = W.w0; w[1] = W.w1; w[2] = W.w2; w[3] = W.w3;
}

}  // namespace gs

// gs_cpuset_dev.h — cpuset selection of NodeNUMAResource Reserve (resourceManager.allocateCPUSet,
// nodenumaresource/resource_manager.go:273-360 -> takeCPUs, cpu_accumulator.go:87-232, and the
// cpuAccumulator list builders :234-822) over core bit planes, so that the commit kernel can Reserve a
// cpuset pod on the device and keep the batch going. The same code is compiled for the host, where the
// library self-test (gsx_cpuset_selftest) compares it with the host restatement (gs_numa_host.cpp take_cpus).
//
// Scope (TopoDev.ok, "compact" topologies): <= 128 cores, <= 8 NUMA nodes and sockets, every core and every NUMA
// node inside one socket, <= 4 CPUs per core up to 64 cores and <= 2 beyond; the node's maxRefCount <= 2 (RefCount
// ordering over one "RefCount 1" plane set). Nodes outside it keep the host path (the commit kernel ends the batch
// after such a pod).
//
// Representation: core rank k = position of the core id in ascending order (the reference's core-id
// tiebreaks), NUMA node / socket index = position of the id in ascending order, CPU position j = rank of
// the CPU id inside its core. A set of CPUs is a set of planes of core masks: plane j, bit k = CPU (k, j) —
// 4 planes of 64-bit masks for <= 64 cores, 2 planes of 128-bit masks beyond (TopoDev.wide). Either way a set is
// 256 bits, stored as 4 packed words (the CPU state columns, the cpuset results); the selection is a template over
// the two shapes, so the common one never carries 128-bit masks in its registers. Lists the reference orders by
// CPU id are materialised as 256-bit CPU masks (cpu_core / cpu_pos map back).
// maxRefCount 2: RC = the available CPUs at RefCount 1; the reference's RefCount orderings (sortCores,
// sortCPUsByRefCount, freeCPUs' core order) become "RefCount-0 CPUs / cores with fewer RefCount-1 CPUs first".
#pragma once
#include <stdint.h>

#include "../../include/gpuscore.h"

#if defined(__HIP__)
#define GS_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define GS_HD inline
#endif
// The topology tables are read-only for a kernel's lifetime: on the device they are read through the constant address
// space, so the wave-uniform reads of the selection below are scalar loads (s_load, through the scalar cache) instead
// of vector loads with a readfirstlane each.
#if defined(__HIP_DEVICE_COMPILE__)
#define GS_TOPO_AS __attribute__((address_space(4)))
#else
#define GS_TOPO_AS
#endif

namespace gs {

constexpr int TD_CORES = 128, TD_NODES = 8, TD_SOCKETS = 8, TD_POS = 4;
typedef unsigned __int128 cm_t;   // a 128-bit core mask (bit k = core rank k)

struct TopoDev {
  int32_t ok;                       // the device path applies to this topology
  int32_t num_cpus, ncores, cpc, cpn, cps, nnodes, nsockets;
  int32_t wide;                     // ncores > 64: 2 planes of 128 cores (cpc <= 2)
  int32_t pad0;
  uint64_t node_cores[TD_NODES][2];     // cores of NUMA node index n (lo, hi word)
  uint64_t sock_cores[TD_SOCKETS][2];   // cores of socket index s
  uint64_t pos_cores[TD_POS][2];        // cores with a CPU at position j
  uint8_t core_node[TD_CORES];
  uint8_t node_sock[TD_NODES];
  uint8_t pad[8];
  uint8_t core_cpu[TD_CORES][TD_POS];
  uint8_t cpu_core[256];
  uint8_t cpu_pos[256];
};
static_assert(sizeof(TopoDev) % 8 == 0, "TopoDev is staged to LDS as 64-bit words");

// Per-node CPU state the device Reserve reads and updates (HBM columns C_CPU_UN0 .. C_CPU_XC1, C_CPU_META). The
// plane sets un / rc are packed words; the layout is the column order of gs_layout.h.
struct CpuStateDev {
  uint64_t un[4];   // not available: RefCount >= maxRefCount, or reserved
  uint64_t xc;      // cores holding an allocated CPU with PCPULevel exclusivity (ranks 0..63)
  uint64_t zal;     // allocated CPUs (RefCount > 0) per zone slot z (16 bits each)
  uint64_t rc[4];   // available CPUs at RefCount 1 (maxRefCount 2; zero otherwise)
  uint64_t xc1;     // xc, ranks 64..127
  uint32_t meta;    // CM_* below
  int32_t topo;     // TopoDev index; -1: cpuset selection stays on the host
};
static_assert(sizeof(CpuStateDev) == 96, "CpuStateDev = 11 i64 columns + meta + topo");
enum : uint32_t {
  CM_XN_MASK = 0xFFu,    // NUMA node indexes holding a NUMANodeLevel-exclusive allocated CPU
  CM_ZIDX_SHIFT = 8,     // 4 x 4 bits: zone slot z -> NUMA node index (0xF: not in the topology)
  CM_MOST = 1u << 24,    // NUMAAllocateStrategy MostAllocated (GetNUMAAllocateStrategy, util.go:35-41)
  CM_MR2 = 1u << 25,     // maxRefCount 2
  CM_XSTALE = 1u << 26,  // xc / xn may be inexact: a CPU of an exclusive node was shared (its policy overwritten)
};

// Wave-uniform reads of the topology / CPU state: on the device these functions run for one Reserve at a time (one
// active lane or identical operands in every lane), so a value read from LDS is moved to a scalar register and the
// selection below runs on the scalar unit instead of one VALU lane.
GS_HD int32_t TU32(int32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_readfirstlane(x);
#else
  return x;
#endif
}
GS_HD uint32_t TUU(uint32_t x) { return (uint32_t)TU32((int32_t)x); }
GS_HD uint64_t TU64(uint64_t x) { return ((uint64_t)TUU((uint32_t)(x >> 32)) << 32) | TUU((uint32_t)x); }
GS_HD uint64_t cm_lo(cm_t x) { return (uint64_t)x; }
GS_HD uint64_t cm_hi(cm_t x) { return (uint64_t)(x >> 64); }

// ---- mask operations for both shapes (M = uint64_t: <= 64 cores, M = cm_t: <= 128)
GS_HD int td_pc(uint64_t x) { return __builtin_popcountll(x); }
GS_HD int td_pc(cm_t x) { return __builtin_popcountll(cm_lo(x)) + __builtin_popcountll(cm_hi(x)); }
GS_HD int td_ctz(uint64_t x) { return __builtin_ctzll(x); }
GS_HD int td_ctz(cm_t x) { return cm_lo(x) ? __builtin_ctzll(cm_lo(x)) : 64 + __builtin_ctzll(cm_hi(x)); }
template <class M> GS_HD M td_tm(const GS_TOPO_AS uint64_t* w);   // a TopoDev mask
template <> GS_HD uint64_t td_tm<uint64_t>(const GS_TOPO_AS uint64_t* w) { return TU64(w[0]); }
template <> GS_HD cm_t td_tm<cm_t>(const GS_TOPO_AS uint64_t* w) { return ((cm_t)TU64(w[1]) << 64) | (cm_t)TU64(w[0]); }
// byte i of a topology table: on the device the aligned dword that holds it (a scalar load; there is no scalar byte
// load on gfx950)
GS_HD int td_u8(const GS_TOPO_AS uint8_t* a, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t w = reinterpret_cast<const GS_TOPO_AS uint32_t*>(a)[i >> 2];
  return (int)((w >> (8 * (i & 3))) & 0xffu);
#else
  return a[i];
#endif
}
template <class M> GS_HD M td_bit(int k) { return (M)1 << k; }
template <class M> GS_HD bool td_has(M x, int k) { return (int)((x >> k) & 1u) != 0; }
template <class M> constexpr int td_bits() { return (int)sizeof(M) * 8; }

template <class M, int NP> GS_HD int td_cnt(const M* P, M m) {
  int n = 0;
#pragma unroll
  for (int j = 0; j < NP; ++j) n += td_pc(P[j] & m);
  return n;
}
template <class M, int NP> GS_HD M td_any(const M* P) {
  M a = 0;
#pragma unroll
  for (int j = 0; j < NP; ++j) a |= P[j];
  return a;
}
template <class M> GS_HD M td_all(const GS_TOPO_AS TopoDev& t) {
  const int n = TU32(t.ncores);
  return n >= td_bits<M>() ? ~(M)0 : (td_bit<M>(n) - 1);
}

// packed words <-> planes
template <class M, int NP> GS_HD void td_unpack(const uint64_t* w, M* P);
template <> GS_HD void td_unpack<uint64_t, 4>(const uint64_t* w, uint64_t* P) {
#pragma unroll
  for (int j = 0; j < 4; ++j) P[j] = TU64(w[j]);
}
template <> GS_HD void td_unpack<cm_t, 2>(const uint64_t* w, cm_t* P) {
  P[0] = ((cm_t)TU64(w[1]) << 64) | TU64(w[0]);
  P[1] = ((cm_t)TU64(w[3]) << 64) | TU64(w[2]);
}
template <class M, int NP> GS_HD void td_pack(const M* P, uint64_t* w);
template <> GS_HD void td_pack<uint64_t, 4>(const uint64_t* P, uint64_t* w) {
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = P[j];
}
template <> GS_HD void td_pack<cm_t, 2>(const cm_t* P, uint64_t* w) {
  w[0] = cm_lo(P[0]); w[1] = cm_hi(P[0]); w[2] = cm_lo(P[1]); w[3] = cm_hi(P[1]);
}

// E[v] = cores with exactly v CPUs set in P (v = 0..4), bit-sliced (planes past NP are empty)
template <class M, int NP> GS_HD void td_exact(const M* P, M* E) {
  const M p2 = NP > 2 ? P[NP > 2 ? 2 : 0] : (M)0, p3 = NP > 3 ? P[NP > 3 ? 3 : 0] : (M)0;
  const M s0 = P[0] ^ P[1], c0 = P[0] & P[1], s1 = p2 ^ p3, c1 = p2 & p3;
  const M b0 = s0 ^ s1, t1 = s0 & s1;
  const M b1 = c0 ^ c1 ^ t1, b2 = (c0 & c1) | (c0 & t1) | (c1 & t1);
  E[0] = ~b0 & ~b1 & ~b2;
  E[1] = b0 & ~b1 & ~b2;
  E[2] = ~b0 & b1 & ~b2;
  E[3] = b0 & b1 & ~b2;
  E[4] = ~b0 & ~b1 & b2;
}
// cores with exactly v CPUs set in P, v a run-time value (no indexed register array: on the device a dynamically
// indexed local array lives in scratch memory)
template <class M, int NP> GS_HD M td_exactly(const M* P, int v) {
  M E[5];
  td_exact<M, NP>(P, E);
  return v == 0 ? E[0] : v == 1 ? E[1] : v == 2 ? E[2] : v == 3 ? E[3] : v == 4 ? E[4] : (M)0;
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

// position of the r-th CPU of core k in P in (RefCount, CPU id) order: the RefCount-0 CPUs (not in RC) by
// position, then the RefCount-1 ones (-1: none)
template <class M, int NP> GS_HD int td_rth(const M* P, const M* RC, int k, int r) {
  for (int pass = 0; pass < 2; ++pass)
#pragma unroll
    for (int j = 0; j < NP; ++j)
      if (td_has(P[j], k) && (int)td_has(RC[j], k) == pass) {
        if (r == 0) return j;
        --r;
      }
  return -1;
}

// cpuAccumulator (cpu_accumulator.go:234-330) with maxRefCount <= 2
template <class M, int NP>
struct DAcc {
  const GS_TOPO_AS TopoDev& t;
  M A[NP];    // allocatableCPUs
  M RC[NP];   // CPUs at RefCount 1 (allocatable or not: only A & RC is read)
  M R[NP];    // result
  M xc;       // exclusiveInCores
  uint32_t xn;   // exclusiveInNUMANodes (node indexes)
  int needed, nalloc, ep;
  bool most, exclusive, refs;

  GS_HD DAcc(const GS_TOPO_AS TopoDev& tt, const M* avail, const M* rc, M xc0, uint32_t xn0, int n, int e, bool m)
      : t(tt), xc(xc0), xn(xn0), needed(n), ep(e), most(m) {
    M any_rc = 0;
#pragma unroll
    for (int j = 0; j < NP; ++j) { A[j] = avail[j]; RC[j] = rc[j]; R[j] = 0; any_rc |= A[j] & RC[j]; }
    refs = any_rc != 0;
    nalloc = td_cnt<M, NP>(A, ~(M)0);
    exclusive = e == GS_CPU_EXCLUSIVE_PCPU_LEVEL || e == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL;
  }
  GS_HD M tm(const GS_TOPO_AS uint64_t* w) const { return td_tm<M>(w); }
  GS_HD bool sless(int a, int b) const { return most ? a < b : a > b; }
  GS_HD int dir(int x) const { return most ? x : 511 - x; }   // ascending key of the sless order
  GS_HD bool satisfied() const { return needed < 1; }
  GS_HD M nodes_cores(uint32_t nodes) const {
    M m = 0;
    for (; nodes; nodes &= nodes - 1) m |= tm(t.node_cores[TU32(__builtin_ctz(nodes))]);
    return m;
  }
  // getCoreRefCount over allocatableCPUs (:776-783): cores whose CPUs in the snapshot S (the allocatable CPUs a list
  // was built from: the reference sorts a list once, before taking from it) hold exactly v at RefCount 1; with no
  // RefCount-1 CPU every core is at level 0
  GS_HD M ref_level(const M* S, int v) const {
    if (!refs) return v == 0 ? ~(M)0 : (M)0;
    M P[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) P[j] = S[j] & RC[j];
    return td_exactly<M, NP>(P, v);
  }
  GS_HD int ref_levels() const { return refs ? NP : 0; }
  // filterExclusive predicates: isCPUExclusivePCPULevel / isCPUExclusiveNUMANodeLevel (:318-330)
  GS_HD M keep_xp(bool fe) const { return (fe && ep == GS_CPU_EXCLUSIVE_PCPU_LEVEL) ? ~xc : ~(M)0; }
  GS_HD M keep_xn(bool fe) const {
    return (fe && ep == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL) ? ~nodes_cores(xn) : ~(M)0;
  }
  GS_HD void take(int k, int j) {   // take (:290-304)
    const M b = td_bit<M>(k);
#pragma unroll
    for (int jj = 0; jj < NP; ++jj) {
      if (jj != j) continue;
      R[jj] |= b;
      if (A[jj] & b) { A[jj] &= ~b; --nalloc; }
    }
    --needed;
    if (exclusive) {
      if (ep == GS_CPU_EXCLUSIVE_PCPU_LEVEL) xc |= b;
      else xn |= 1u << td_u8(t.core_node, TU32(k));
    }
  }
  // the first `n` allocatable CPUs of core k in CPU order
  GS_HD void take_core(int k, int n) {
#pragma unroll
    for (int j = 0; j < NP; ++j)
      if (n > 0 && td_has(A[j], k)) { take(k, j); --n; }
  }
  // head(list, needed) of a full-core list: cores by (RefCount asc, id) (sortCores, :345-367), CPUs ascending
  GS_HD void take_head_cores(M q) {
    const int nl = ref_levels();
    M S[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) S[j] = A[j];
    for (int v = 0; v <= nl && needed > 0; ++v)
      for (M b = q & ref_level(S, v); b && needed > 0; b &= b - 1)
        take_core(td_ctz(b), needed < TU32(t.cpc) ? needed : TU32(t.cpc));
  }
  // Takes up to `needed` CPUs, in (RefCount, CPU id) order, out of the pass-r CPUs (the r-th CPU of each core in
  // (RefCount, id) order) of the snapshot S; r < 0: all CPUs of S.
  GS_HD void take_cpu_order(const M* S, int r) {
    TdMask256 W0, W1;   // RefCount 0 / 1
    for (M b = td_any<M, NP>(S); b; b &= b - 1) {
      const int k = td_ctz(b);
      const int jr = r >= 0 ? td_rth<M, NP>(S, RC, k, r) : -1;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        if (!td_has(S[j], k) || (r >= 0 && j != jr)) continue;
        const int c = td_u8(&t.core_cpu[0][0], TU32(k) * TD_POS + TU32(j));
        if (td_has(RC[j], k)) W1.set_bit(c);
        else W0.set_bit(c);
      }
    }
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const TdMask256& W = g ? W1 : W0;
        for (uint64_t x = w == 0 ? W.w0 : w == 1 ? W.w1 : w == 2 ? W.w2 : W.w3; x && needed > 0; x &= x - 1) {
          const int c = w * 64 + __builtin_ctzll(x);
          take(td_u8(t.cpu_core, TU32(c)), td_u8(t.cpu_pos, TU32(c)));
        }
      }
  }
  // head(spreadCPUs(list), needed) for a list in (RefCount, CPU id) order (sortCPUsByRefCount, :785-797): the CPUs
  // of cores `m` in A; `first_only`: the list went through extractCPU (one CPU per core), L = its length
  GS_HD void take_spread_cpu_list(M m, bool first_only, int L) {
    M S[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) S[j] = A[j] & m;
    if (!first_only && L <= TU32(t.cpc)) { take_cpu_order(S, -1); return; }   // spreadCPUs keeps short lists as is
    const int passes = first_only ? 1 : NP;
    for (int r = 0; r < passes && needed > 0; ++r) take_cpu_order(S, r);
  }
  GS_HD M full_cores(M keep) const {
    M K[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) K[j] = A[j] & keep;
    return td_exactly<M, NP>(K, TU32(t.cpc)) & td_any<M, NP>(K);
  }
  // freeCoresInNode(true, fe) (:370-461): the first NUMA node list with >= needed CPUs (-1: none)
  GS_HD int pick_full_node(bool fe, M* cores) const {
    const M keep = td_all<M>(t) & keep_xn(fe);
    const M full = full_cores(keep);
    int best = -1, bsz = 0, bsf = 0;
    for (int n = 0; n < TU32(t.nnodes); ++n) {
      const M q = full & tm(t.node_cores[TU32(n)]);
      if (!q) continue;
      const int sz = TU32(t.cpc) * td_pc(q);
      if (sz < needed) continue;
      const int sf = td_cnt<M, NP>(A, keep & tm(t.sock_cores[td_u8(t.node_sock, TU32(n))]));
      if (best < 0 || sless(sz, bsz) || (sz == bsz && sless(sf, bsf))) { best = n; bsz = sz; bsf = sf; *cores = q; }
    }
    return best;
  }
  // freeCoresInSocket(true) (:463-527): the first socket list with >= needed CPUs
  GS_HD int pick_full_socket(M* cores) const {
    const M full = full_cores(~(M)0);
    int best = -1, bsz = 0;
    for (int s = 0; s < TU32(t.nsockets); ++s) {
      const M q = full & tm(t.sock_cores[TU32(s)]);
      if (!q) continue;
      const int sz = TU32(t.cpc) * td_pc(q);
      if (sz < needed) continue;
      if (best < 0 || sless(sz, bsz)) { best = s; bsz = sz; *cores = q; }
    }
    return best;
  }
  // freeCPUsInNode(fe) (:529-605) / freeCPUsInSocket(fe) (:607-656): the first list with >= needed CPUs
  GS_HD int pick_cpus(bool node, bool fe, M* cores, int* L) const {
    const M keep = td_all<M>(t) & keep_xp(fe) & (node ? keep_xn(fe) : ~(M)0);
    int best = -1, bnf = 0, bsf = 0;
    const int cnt = node ? TU32(t.nnodes) : TU32(t.nsockets);
    for (int n = 0; n < cnt; ++n) {
      const M m = keep & tm(node ? t.node_cores[TU32(n)] : t.sock_cores[TU32(n)]);
      const int nf = td_cnt<M, NP>(A, m);
      if (nf == 0) continue;
      const int len = fe ? td_pc(td_any<M, NP>(A) & m) : nf;
      if (len < needed) continue;
      if (node) {   // NUMA nodes by (free CPUs, socket free CPUs, id)
        const int sf = td_cnt<M, NP>(A, keep & tm(t.sock_cores[td_u8(t.node_sock, TU32(n))]));
        if (best < 0 || sless(nf, bnf) || (nf == bnf && sless(sf, bsf))) {
          best = n; bnf = nf; bsf = sf; *cores = m; *L = len;
        }
      } else if (best < 0 || sless(len, bnf)) {   // sockets by (list length, id)
        best = n; bnf = len; *cores = m; *L = len;
      }
    }
    return best;
  }
  // head(spreadCPUs(freeCPUs(fe)), needed) (:658-774): cores ordered by (CPUs of the result in the socket
  // desc, socket free, node free, core size asc, socket id, core RefCount asc, core id), CPUs of a core in
  // (RefCount, id) order
  GS_HD void take_free_cpus(bool fe) {
    const M keep = td_all<M>(t) & keep_xp(fe) & keep_xn(fe);
    M S[NP], E[5];
#pragma unroll
    for (int j = 0; j < NP; ++j) S[j] = A[j] & keep;
    const M cores = td_any<M, NP>(S);
    if (!cores) return;
    td_exact<M, NP>(S, E);
    const int L = td_cnt<M, NP>(S, ~(M)0);
    const int nl = ref_levels();
    // NUMA nodes by group key (colo desc, socket free, node free), ascending; equal keys merge
    // entry i = (key << 3 | node) of the i-th node in key order (stable)
    TdPack8 ok;
    int nn = 0;
    for (int n = 0; n < TU32(t.nnodes); ++n) {
      if (!(cores & tm(t.node_cores[TU32(n)]))) continue;
      const M sm = tm(t.sock_cores[td_u8(t.node_sock, TU32(n))]);
      const int colo = td_cnt<M, NP>(R, sm), sf = td_cnt<M, NP>(S, sm), nf = td_cnt<M, NP>(S, tm(t.node_cores[TU32(n)]));
      const uint32_t kn = ((uint32_t)(511 - colo) << 18) | ((uint32_t)dir(sf) << 9) | (uint32_t)dir(nf);
      int i = nn++;   // insertion after the last key <= kn (stable)
      while (i > 0 && (ok.get(i - 1) >> 3) > kn) { ok.set(i, ok.get(i - 1)); --i; }
      ok.set(i, kn << 3 | (uint32_t)n);
    }
    const bool as_is = L <= TU32(t.cpc);   // spreadCPUs keeps short lists as is
    const int passes = as_is ? 1 : NP;
    for (int r = 0; r < passes; ++r) {
      for (int g = 0; g < nn;) {
        M Mg = 0;
        int h = g;
        const uint32_t kg = ok.get(g) >> 3;
        for (; h < nn && (ok.get(h) >> 3) == kg; ++h) Mg |= cores & tm(t.node_cores[TU32(ok.get(h) & 7u)]);
        g = h;
#pragma unroll
        for (int v = 1; v <= NP; ++v) {
          if (!as_is && v <= r) continue;
          const M Mv = Mg & E[v];
          if (!Mv) continue;
          for (int s = 0; s < TU32(t.nsockets); ++s)
            for (int rl = 0; rl <= nl; ++rl)
              for (M q = Mv & tm(t.sock_cores[TU32(s)]) & ref_level(S, rl); q; q &= q - 1) {
                const int k = td_ctz(q);
                if (as_is) {
                  for (int pass = 0; pass < 2 && needed > 0; ++pass)
#pragma unroll
                    for (int j = 0; j < NP; ++j)
                      if (needed > 0 && td_has(S[j], k) && (int)td_has(RC[j], k) == pass) take(k, j);
                } else {
                  take(k, td_rth<M, NP>(S, RC, k, r));
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

// takeCPUs (cpu_accumulator.go:87-232); avail = planes of the CPUs it may take, rc = the RefCount-1 planes.
// false: the reference errors.
template <class M, int NP>
GS_HD bool td_take_cpus_t(const GS_TOPO_AS TopoDev& t, const M* avail, const M* rc, M xc, uint32_t xn, int needed, int bind,
                          int ep, bool most, M* out) {
  DAcc<M, NP> a(t, avail, rc, xc, xn, needed, ep, most);
#pragma unroll
  for (int j = 0; j < NP; ++j) out[j] = 0;
  if (a.satisfied()) return true;
  if (a.needed > a.nalloc) return false;
  const bool full = bind == GS_CPU_BIND_FULL_PCPUS;
  bool ok = false;
  do {
    M m = 0;
    int L = 0;
    if (full || TU32(t.cpc) == 1) {
      bool got = false;
      for (int fe = 1; fe >= 0 && !got && a.needed <= TU32(t.cpn); --fe) got = a.pick_full_node(fe != 0, &m) >= 0;
      if (!got && a.needed <= TU32(t.cps)) got = a.pick_full_socket(&m) >= 0;
      if (got) {
        a.take_head_cores(m);
        ok = true;
        break;
      }
      // freeCoresInSocket(true) in (size, id) order, then sort.Slice by size desc (:141-155)
      const M fc = a.full_cores(~(M)0);
      TdPack8 so;   // (size << 3 | socket index)
      int ns = 0;
      for (int s = 0; s < TU32(t.nsockets); ++s) {
        const M q = fc & a.tm(t.sock_cores[TU32(s)]);
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
        for (M b = fc & a.tm(t.sock_cores[TU32(idi)]); b; b &= b - 1) a.take_core(td_ctz(b), TD_POS);
        ok = a.satisfied();
      }
      if (ok) break;
      if (a.needed >= TU32(t.cpc)) {   // (:157-176): the lists' cores in (RefCount, id) order, cpc CPUs at a time
        td_go_sort(uo, nu, false);
        const int nl = a.ref_levels();
        for (int i = 0; i < nu && !ok; ++i) {
          const M sc = fc & a.tm(t.sock_cores[TU32(uo.get(i) & 7u)]);
          M S[NP];
#pragma unroll
          for (int j = 0; j < NP; ++j) S[j] = a.A[j];
          bool brk = false;
          for (int v = 0; v <= nl && !brk; ++v)
            for (M b = sc & a.ref_level(S, v); b; b &= b - 1) {
              a.take_core(td_ctz(b), TD_POS);
              if (a.satisfied()) { ok = true; brk = true; break; }
              if (a.needed < TU32(t.cpc)) { brk = true; break; }
            }
        }
        if (ok) break;
      }
    }
    if (!full) {   // (:184-215): node lists (filterExclusive true, false), then socket lists; one call site of each
      int found = -1;   // (a run-time loop keeps one inlined copy of the list code)
      for (int k = 0; k < 4 && found < 0; ++k) {
        const bool node = k < 2;
        if (a.needed > (node ? TU32(t.cpn) : TU32(t.cps))) continue;
        if (a.pick_cpus(node, (k & 1) == 0, &m, &L) >= 0) found = k;
      }
      if (found >= 0) { a.take_spread_cpu_list(m, (found & 1) == 0, L); ok = true; break; }
    }
    for (int fe = 1; fe >= 0 && !ok; --fe) {   // (:217-229)
      a.take_free_cpus(fe != 0);
      ok = a.satisfied();
    }
  } while (false);
  if (!ok) return false;
#pragma unroll
  for (int j = 0; j < NP; ++j) out[j] = a.R[j];
  return true;
}

template <class M> GS_HD M td_xc(const CpuStateDev& cs);
template <> GS_HD uint64_t td_xc<uint64_t>(const CpuStateDev& cs) { return TU64(cs.xc); }
template <> GS_HD cm_t td_xc<cm_t>(const CpuStateDev& cs) { return ((cm_t)TU64(cs.xc1) << 64) | (cm_t)TU64(cs.xc); }
GS_HD int td_zone_node(const CpuStateDev& cs, int z) { return (int)((TUU(cs.meta) >> (CM_ZIDX_SHIFT + 4 * z)) & 15u); }

// available CPUs (getAvailableCPUs, node_allocation.go:142-162: RefCount < maxRefCount, not reserved) as planes
template <class M, int NP> GS_HD void td_available(const GS_TOPO_AS TopoDev& t, const CpuStateDev& cs, M* P) {
  M U[NP];
  td_unpack<M, NP>(cs.un, U);
#pragma unroll
  for (int j = 0; j < NP; ++j) P[j] = td_tm<M>(t.pos_cores[TU32(j)]) & ~U[j];
}

// allocateCPUSet (resource_manager.go:273-360) given the NUMA split Allocate produced (PlacementDev zkeys /
// zcpu), the cpuset as packed words. false: the reference errors (cannot follow a feasible Filter; the host fails
// loudly).
template <class M, int NP>
GS_HD bool td_allocate_cpuset_t(const GS_TOPO_AS TopoDev& t, const CpuStateDev& cs, int num_cpus, int bind, bool required, int ep,
                                uint32_t zkeys, const int64_t* zcpu, uint64_t* out_w) {
  M P[NP], RC[NP], out[NP];
  td_available<M, NP>(t, cs, P);
  td_unpack<M, NP>(cs.rc, RC);
  const bool most = TUU(cs.meta) & CM_MOST;
  const M xc = td_xc<M>(cs);
  const uint32_t xn = TUU(cs.meta) & CM_XN_MASK;
  if (required) {   // filterCPUsByRequiredCPUBindPolicy (:534-566)
    if (bind == GS_CPU_BIND_FULL_PCPUS) {
      const M f = td_exactly<M, NP>(P, TU32(t.cpc)) & td_any<M, NP>(P);
#pragma unroll
      for (int j = 0; j < NP; ++j) P[j] &= f;
    } else if (bind == GS_CPU_BIND_SPREAD_BY_PCPUS) {
      M seen = 0;
#pragma unroll
      for (int j = 0; j < NP; ++j) { P[j] &= ~seen; seen |= P[j]; }
    }
  }
#pragma unroll
  for (int j = 0; j < NP; ++j) out[j] = 0;
  for (int j = 0; j < 4; ++j) out_w[j] = 0;
  if (td_cnt<M, NP>(P, ~(M)0) < num_cpus) return false;
  // takePreferredCPUs per hinted zone (zkeys: the NUMA split), or once over every available CPU; one call site of
  // the selection (a second inlined copy doubles the function's registers)
  for (int z = zkeys ? 0 : 4; z < (zkeys ? 4 : 5); ++z) {
    M in[NP];
    int num = num_cpus;
    if (z < 4) {
      if (!((zkeys >> z) & 1u) && !((zkeys >> (4 + z)) & 1u)) continue;
      const int n = td_zone_node(cs, z);
      const M m = n < TU32(t.nnodes) ? td_tm<M>(t.node_cores[TU32(n)]) : (M)0;
#pragma unroll
      for (int j = 0; j < NP; ++j) in[j] = P[j] & m;
      num = td_cnt<M, NP>(in, ~(M)0);
      const int64_t zz = z == 0 ? zcpu[0] : z == 1 ? zcpu[1] : z == 2 ? zcpu[2] : zcpu[3];
      const int want = ((zkeys >> z) & 1u) ? (int)(zz / 1000) : 0;
      if (want < num) num = want;
      if (num <= 0) continue;   // takePreferredCPUs with nothing needed
    } else {
#pragma unroll
      for (int j = 0; j < NP; ++j) in[j] = P[j];
    }
    M got[NP];
    if (!td_take_cpus_t<M, NP>(t, in, RC, xc, xn, num, bind, ep, most, got)) return false;
#pragma unroll
    for (int j = 0; j < NP; ++j) out[j] |= got[j];
  }
  if (zkeys && td_cnt<M, NP>(out, ~(M)0) != num_cpus) return false;
  if (required) {   // satisfiedRequiredCPUBindPolicy (:568-589)
    const int nc = td_pc(td_any<M, NP>(out)), ncpus = td_cnt<M, NP>(out, ~(M)0);
    if (bind == GS_CPU_BIND_FULL_PCPUS && nc * TU32(t.cpc) != ncpus) return false;
    if (bind == GS_CPU_BIND_SPREAD_BY_PCPUS && nc != ncpus) return false;
  }
  td_pack<M, NP>(out, out_w);
  return true;
}

// NodeAllocation.addPodAllocation (node_allocation.go:77-96) of the cpuset R (packed words) with exclusive policy ep
// on the CPU state: RefCount + 1 on every CPU of R (maxRefCount 1: they leave the available set; 2: those already at
// RefCount 1 do, the others move to RefCount 1), the exclusive cores / NUMA nodes, the allocated CPUs per zone slot
// (nz slots). Every CPU of R takes ep as its ExclusivePolicy; when a CPU already allocated is shared on a node with
// exclusive CPUs, the policy it loses is not known here, and xc / xn are marked stale (CM_XSTALE: a later pod whose
// selection reads them leaves the device path). Returns the number of newly allocated CPUs (RefCount 0 -> 1).
template <class M, int NP>
GS_HD int td_reserve_update_t(const GS_TOPO_AS TopoDev& t, CpuStateDev& cs, const uint64_t* R_w, int ep, int nz) {
  M U[NP], RC[NP], R[NP], NEW[NP];
  td_unpack<M, NP>(cs.un, U);
  td_unpack<M, NP>(cs.rc, RC);
  td_unpack<M, NP>(R_w, R);
  uint32_t meta = TUU(cs.meta);
  const bool mr2 = meta & CM_MR2;
  M shared = 0;
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    NEW[j] = R[j] & ~RC[j];
    shared |= R[j] & RC[j];
    if (mr2) {
      U[j] |= R[j] & RC[j];
      RC[j] ^= R[j];
    } else {
      U[j] |= R[j];
    }
  }
  M xc = td_xc<M>(cs);
  if (shared && (xc || (meta & CM_XN_MASK))) meta |= CM_XSTALE;
  const M cores = td_any<M, NP>(R);
  if (ep == GS_CPU_EXCLUSIVE_PCPU_LEVEL) xc |= cores;
  else if (ep == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL)
    for (M b = cores; b; b &= b - 1) meta |= 1u << td_u8(t.core_node, TU32(td_ctz(b)));
  uint64_t zal = TU64(cs.zal);
  for (int z = 0; z < 4; ++z) {
    const int n = td_zone_node(cs, z);
    if (z >= nz || n >= TU32(t.nnodes)) continue;   // a zone the topology lacks keeps its zero summaries
    const uint64_t zc = ((zal >> (16 * z)) & 0xFFFFull) + (uint64_t)td_cnt<M, NP>(NEW, td_tm<M>(t.node_cores[TU32(n)]));
    zal = (zal & ~(0xFFFFull << (16 * z))) | (zc << (16 * z));
  }
  td_pack<M, NP>(U, cs.un);
  td_pack<M, NP>(RC, cs.rc);
  const cm_t x128 = (cm_t)xc;
  cs.xc = cm_lo(x128);
  cs.xc1 = cm_hi(x128);
  cs.zal = zal;
  cs.meta = meta;
  return td_cnt<M, NP>(NEW, ~(M)0);
}

// available-CPU counts of NUMA node index n (-1: every node): raw | full-core CPUs << 9 | cores with a free CPU
// << 18, packed as gs_numa_host.cpp count_available
template <class M, int NP> GS_HD int32_t td_counts_t(const GS_TOPO_AS TopoDev& t, const CpuStateDev& cs, int n) {
  M P[NP];
  td_available<M, NP>(t, cs, P);
  const M m = n < 0 ? ~(M)0 : td_tm<M>(t.node_cores[TU32(n)]);
#pragma unroll
  for (int j = 0; j < NP; ++j) P[j] &= m;
  const int raw = td_cnt<M, NP>(P, ~(M)0);
  const int full = TU32(t.cpc) * td_pc(td_exactly<M, NP>(P, TU32(t.cpc)) & td_any<M, NP>(P));
  const int spread = td_pc(td_any<M, NP>(P));
  return (int32_t)(raw | (full << 9) | (spread << 18));
}

// the cpuset (packed words) as a 256-bit CPU mask
template <class M, int NP> GS_HD void td_to_cpus_t(const GS_TOPO_AS TopoDev& t, const uint64_t* R_w, uint64_t* w) {
  M R[NP];
  td_unpack<M, NP>(R_w, R);
  TdMask256 W;
#pragma unroll
  for (int j = 0; j < NP; ++j)
    for (M b = R[j]; b; b &= b - 1) W.set_bit(td_u8(&t.core_cpu[0][0], TU32(td_ctz(b)) * TD_POS + TU32(j)));
  w[0] = W.w0; w[1] = W.w1; w[2] = W.w2; w[3] = W.w3;
}

// the topology as the selection reads it (the constant address space on the device)
GS_HD const GS_TOPO_AS TopoDev& td_topo(const TopoDev& t) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const GS_TOPO_AS TopoDev*)(uint64_t)&t;
#else
  return t;
#endif
}

// ---- the packed-word API: the shape is the topology's (TopoDev.wide)
GS_HD bool td_allocate_cpuset(const TopoDev& tg, const CpuStateDev& cs, int num_cpus, int bind, bool required, int ep,
                              uint32_t zkeys, const int64_t* zcpu, uint64_t* out_w) {
  const GS_TOPO_AS TopoDev& t = td_topo(tg);
  return TU32(t.wide) ? td_allocate_cpuset_t<cm_t, 2>(t, cs, num_cpus, bind, required, ep, zkeys, zcpu, out_w)
                      : td_allocate_cpuset_t<uint64_t, 4>(t, cs, num_cpus, bind, required, ep, zkeys, zcpu, out_w);
}
GS_HD int td_reserve_update(const TopoDev& tg, CpuStateDev& cs, const uint64_t* R_w, int ep, int nz) {
  const GS_TOPO_AS TopoDev& t = td_topo(tg);
  return TU32(t.wide) ? td_reserve_update_t<cm_t, 2>(t, cs, R_w, ep, nz)
                      : td_reserve_update_t<uint64_t, 4>(t, cs, R_w, ep, nz);
}
GS_HD int32_t td_counts(const TopoDev& tg, const CpuStateDev& cs, int n) {
  const GS_TOPO_AS TopoDev& t = td_topo(tg);
  return TU32(t.wide) ? td_counts_t<cm_t, 2>(t, cs, n) : td_counts_t<uint64_t, 4>(t, cs, n);
}
GS_HD void td_to_cpus(const TopoDev& tg, const uint64_t* R_w, uint64_t* w) {
  const GS_TOPO_AS TopoDev& t = td_topo(tg);
  if (TU32(t.wide)) td_to_cpus_t<cm_t, 2>(t, R_w, w);
  else td_to_cpus_t<uint64_t, 4>(t, R_w, w);
}
// takeCPUs over the available CPUs of the state (the self-test's entry; the device selects through allocateCPUSet)
GS_HD bool td_take_cpus(const TopoDev& tg, const CpuStateDev& cs, int needed, int bind, int ep, bool most,
                        uint64_t* out_w) {
  const GS_TOPO_AS TopoDev& t = td_topo(tg);
  for (int j = 0; j < 4; ++j) out_w[j] = 0;
  if (TU32(t.wide)) {
    cm_t P[2], RC[2], R[2];
    td_available<cm_t, 2>(t, cs, P);
    td_unpack<cm_t, 2>(cs.rc, RC);
    if (!td_take_cpus_t<cm_t, 2>(t, P, RC, td_xc<cm_t>(cs), TUU(cs.meta) & CM_XN_MASK, needed, bind, ep, most, R))
      return false;
    td_pack<cm_t, 2>(R, out_w);
  } else {
    uint64_t P[4], RC[4], R[4];
    td_available<uint64_t, 4>(t, cs, P);
    td_unpack<uint64_t, 4>(cs.rc, RC);
    if (!td_take_cpus_t<uint64_t, 4>(t, P, RC, td_xc<uint64_t>(cs), TUU(cs.meta) & CM_XN_MASK, needed, bind, ep,
                                     most, R))
      return false;
    td_pack<uint64_t, 4>(R, out_w);
  }
  return true;
}

}  // namespace gs

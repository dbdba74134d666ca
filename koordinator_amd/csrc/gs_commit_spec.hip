// gs_commit_spec.hip — the sequential commit of a batch as a speculative pipeline on one CU (gfx950, one shard).
//
// Same contract and results as commit_kernel (gs_kernels.hip): the batch's pods in queue order, each one
// selectHost over its batch-start score levels and the rows earlier pods of the batch landed on ("dirty" rows,
// re-scored exactly), then assume + Reserve ([upstream] scheduleOne: selectHost, assume; LoadAware /
// NodeNUMAResource Reserve).
//
// Why speculative. One wave issues about one instruction per 4-8 cycles, and the exact chain per pod — selection,
// Reserve of the winner, the winner row's new score for the next pod — is several thousand instructions long. The
// new score is only needed to know whether the row the previous pod landed on competes again; it rarely does (the
// row just lost capacity). So the selection of pod q runs as soon as pod q-1 is decided, with the rows whose new
// scores are not yet known ("pending") left out, and is verified once they are: pod q stands iff every pending
// row's exact score for q is below q's maximum M_q (then its Feasible count gains the pending rows that are
// feasible). Otherwise the pipeline rolls back to q (undo log of the Reserves after it) and decides q again with
// every score exact. Verified decisions are exactly those of the sequential loop.
//
// Roles (8 waves; wave w runs on SIMD w % 4, see sp_reserve_index / sp_rescore_index below):
//   wave 0       decide (selectHost over levels + ready dirty rows, pending rows excluded), in order; performs the
//                rollbacks the verifier requests. Highest issue priority: it sets the pipeline's pace.
//   wave 4       verify the decisions in order (pending rows' exact re-scores below the decided maximum), the final
//                Feasible counts, and the batch's end; a miss requests a rollback from wave 0. (SIMD 0, beside the
//                selector: the lightest role.)
//   waves 2, 3   Reserve of decided pods, wave 2 the even pods and wave 3 the odd ones: fetch a fresh winner row into
//                its slot (prefetched one pod of its parity ahead), log the slot's state, apply assume + Reserve (NUMA
//                split, cpuset), queue the row's re-scoring on the wave's own job ring. A pod landing on a row an
//                earlier pod landed on waits until that version is re-scored (so the other wave's Reserve is in).
//   waves 1, 5, 6, 7  re-scoring jobs from both rings: a reserved row's new score for 64 later pods, one pod per lane
//                (each wave builds the row's hint table itself).
// Split selector (SPLIT, the default for one shard): the decision is two waves.
//   wave 1       prep: selectHost of pod p over a snapshot of the decisions published so far (s_snap, the slot table
//                in LDS), at most one pod ahead of wave 0, into a PrepRec (M, T, F, tie-break position, the next
//                SP_KW ties in node order, per-slot ready / feasible / tie / pending flags); on request it records a
//                pod again over the exact state (full-row and forced decisions, stops, anything wave 0 cannot patch).
//   wave 0       applies the decisions made after the snapshot (landed slots lose their exact score / were clean
//                nodes to the prep wave: ties excluded and re-ranked in the window, feasibility out of F), settles
//                pending rows whose re-scoring has finished, records the decision, verifies the decided pods in order
//                (no verify wave) and performs the rollbacks.
//   waves 4-7    re-scoring; waves 2, 3 Reserve as above.
// All hand-offs are LDS words (release / acquire); every wait is bounded: an expired wait (any wave) ends the kernel
// with a site code in committed[3], nothing committed and nothing written back (the host fails the call with
// GS_EDEVICE; HBM and host mirror both keep the batch-start state), so a bug cannot hang the GPU.
//
// Several shards (a.nranks > 1): the levels are the all-gathered shards' levels merged into one list per pod
// (merge_levels_kernel), and every rank runs this kernel on them over its full mirror replica. A fresh winner row
// outside the rank's shard has no batch-start score row here (S_own is the own shard's), so its batch-start scores
// for the later pods are unknown (SO_UNKNOWN in dso) until a re-scoring wave has evaluated the row as it stood at
// batch start (the HBM mirror: rows are written back at the kernel's end) — a "batch-start job" queued by the
// Reserve wave. Meanwhile a decision finds such a node in the pod's list head (its listed level: exact), or records
// it as unknown: the decision treated the node as clean and unlisted, which stands iff its batch-start score turns
// out below the decided maximum; the verification checks that (and takes the node's batch-start feasibility out of
// the Feasible count) once the creating pod is complete — same rule as a pending row.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_eval_dev.h"

namespace gs {

constexpr int SP_WAVES = 8, SP_THREADS = 64 * SP_WAVES;
constexpr int SP_LAG = 12;       // decided - verified <= SP_LAG (undo log depth)
constexpr int SP_RES0 = 2, SP_NRES = 2;   // Reserve waves 2, 3 (pod parity)
constexpr int SP_RS0 = SP_RES0 + SP_NRES, SP_TABLES = SP_WAVES - SP_RS0;   // re-scoring waves, one hint table each
// Role -> wave index. The CU runs wave w on SIMD w % 4, two waves per SIMD: the selector (wave 0) shares its SIMD with
// the verifier, the lightest role, instead of a busy re-scoring wave; the Reserve and re-scoring waves fill SIMDs 1-3.
constexpr int SP_W_VERIFY = 4;
__device__ __forceinline__ int sp_reserve_index(int wv) { return wv == 2 ? 0 : wv == 3 ? 1 : -1; }
__device__ __forceinline__ int sp_rescore_index(int wv) { return wv == 1 ? 0 : wv >= 5 ? wv - 4 : -1; }
constexpr int SP_JOBQ = 24;      // job ring per Reserve wave (<= 3 jobs per pod, <= SP_LAG / 2 + 2 pods in flight)
constexpr int SP_HASH = 128;     // node -> slot (full-row resolution; <= MAX_BATCH slots, linear probing)
static_assert(SP_HASH >= MAX_BATCH && (SP_HASH & (SP_HASH - 1)) == 0,
              "the node -> slot hash must hold every dirty slot (its insertion probes until a free entry)");
constexpr int SP_FRESH = 1, SP_FITERR = 2, SP_SLOW = 4, SP_OFFSHARD = 8;   // DecRec.flags
constexpr int SP_PRED_GE = 16, SP_PRED_GT = 32;   // diagnostics (ST): a pending row's pre-landing score >= / > M
constexpr uint32_t SP_SPIN_LIMIT = 1u << 24;
constexpr int SP_NST = 62, SP_STRIDE = 64;   // diagnostics: stamps per wave, the wave's region in a.stamps
constexpr int16_t SO_UNKNOWN = -2;    // dso: batch-start score of an off-shard fresh row not evaluated yet
constexpr int16_t SO_UNLISTED = -3;   // a decision's view of such a row not in the pod's list head

struct DecRec {          // one decided pod
  int32_t winner;        // node (-1: FitError)
  int32_t slot;          // dirty slot it lands on
  int32_t M, T, F;       // max score, ties, feasible count with the pending rows left out
  int32_t nd_before;     // dirty slots before this decision
  int32_t prev_pend;     // the slot's previous version (a landing on an existing slot)
  uint32_t flags;
  uint64_t pend0, pend1; // pending slots at decision time
  uint64_t unk0, unk1;   // slots whose batch-start score was unknown at decision time (several shards)
};
struct UndoRec {         // a slot's state before a Reserve
  Row row;
  CpuStateDev cs;
  int32_t slot, pad;
};
struct Job {
  int32_t slot, q, range, tbl;
};
// the split pipeline (SPLIT): the prep wave's provisional decision of pod p for wave 0
constexpr int SP_KW = 4;          // ties recorded from the tie-break position on (the window wave 0 re-ranks in)
constexpr int SP_PREPQ = 3;       // PrepRec ring: the prep wave works at most SP_PREPQ - 1 pods ahead of wave 0
constexpr int SP_W_PREP = 1;      // its wave (SIMD 1; wave 0 decides on SIMD 0)
struct PrepRec {                    // (the first 80 bytes read as five 16-byte words)
  int32_t pod, q_s, nd_s, action;   // q_s: decisions in the snapshot (nd_s slots); action 0, 1 (FitError), 2 (stop),
                                    // 5: only over the exact state (q_s == pod)
  int32_t M, Mclean, F, ntw;        // ntw: ties in tw
  int32_t end_why, slow;            // action 2 (stop; exact snapshots only): why; slow: forced / full-row decision
  int32_t T_lo, T_hi, jp_lo, jp_hi, pad0, pad1;
  uint32_t tw[SP_KW];               // the ties ranked jp, jp+1, ... (node ids)
  uint8_t sf[MAX_BATCH];            // per snapshot slot: SF_* flags
};
constexpr int SF_READY = 1, SF_FEAS = 2, SF_TIE = 4, SF_PEND = 8;   // ready (exact score counted), ... feasible, ... at
                                                                     // M; pending (left out)
struct Hdr {             // a pod's level header and list head, one value per lane (load_hdr)
  int hs, hc, nlev, feas, next;
  uint32_t lh;
  int32_t tbv;
};
struct Dc {              // a decision before it is recorded (decide_core)
  int action, end_why;   // 0 commit, 1 FitError, 2 stop before the pod, 3 full-row resolution, 4 wait (diagnostics)
  uint32_t winner;
  int M, F, Mclean, Md, Fd;
  int64_t T, jp;
  bool slowpath;
  uint64_t pend0, pend1, unk0, unk1;
  int sc0, sc1, so0, so1;            // per lane: slot lane / lane + 64
  int sf0, sf1;                      // prep wave, per lane: slot lane / lane + 64's SF_* flags
  uint32_t twv;                      // prep wave: tie jp + k in lane k
  int ntw;
};
template <bool B_>
struct Tag {
  static constexpr bool v = B_;
};

__device__ __forceinline__ void sp_sleep() { __builtin_amdgcn_s_sleep(2); }
__device__ __forceinline__ void sp_prio(uint32_t p) {   // s_setprio takes an immediate
  if (p == 1) __builtin_amdgcn_s_setprio(1);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p == 3) __builtin_amdgcn_s_setprio(3);
}

// The kernel's LDS, at fixed offsets sized for MAX_BATCH pods whatever the batch: every array is at a link-time
// constant address and [pod][slot] rows have the constant stride SB, so no register holds a carve-up pointer and
// index arithmetic is a shift (the selector wave is instruction-bound; the carve-up pointers used to be SGPRs spilled
// to VGPR lanes).
constexpr int SB = MAX_BATCH;
struct alignas(16) SpecLds {
  alignas(16) unsigned char pods_b[SB * POD_STRIDE];
  alignas(16) Row drows[SB];                 // dirty rows
  alignas(16) int16_t dsc[SB * SB];          // [pod][slot] current score
  alignas(16) int16_t dso[SB * SB];          // [pod][slot] batch-start score
  alignas(16) CpuStateDev cst[SB];           // cpu state of the dirty rows
  alignas(16) DecRec dec[SB];
  alignas(16) UndoRec undo[SP_LAG];
  alignas(16) HintTable tables[SP_TABLES];
  alignas(16) int32_t final_F[SB], done_ver[SB], has_row[SB], rescored[SB], jobs_left[SB], jobs_all[SB], resv[SB];
  alignas(16) int32_t hkey[SP_HASH];
  alignas(16) int16_t hval[SP_HASH];   // slot of the node in hkey
  alignas(16) Job jobq[SP_NRES * SP_JOBQ];
  alignas(16) PrepRec prq[SP_PREPQ];       // split pipeline: the prep wave's records
  alignas(16) int32_t slot_node[SB];   // split pipeline: the slot table the prep wave snapshots
  alignas(16) int16_t slot_pv[SB];
};

size_t spec_smem_bytes(int) { return sizeof(SpecLds); }
// the CU's 160 KiB hold SpecLds and the kernel's static __shared__ words (~200 B of hand-off words)
static_assert(sizeof(SpecLds) + 200 <= 160 * 1024, "commit_spec_kernel LDS over the CU's 160 KiB");

// LDS hand-off words between the roles (namespace scope: the role functions below and the kernel share them)
__shared__ uint64_t s_cpuset[SP_NRES][4];
__shared__ int32_t s_aff[SP_NRES];
// the four words the selector checks before every decision, adjacent: one 128-bit LDS read (ld_ctl) instead of four
// dependent acquire loads
__shared__ __attribute__((aligned(16))) int32_t s_ctl[4];
#define s_rb_req s_ctl[0]     // verifier -> wave 0: v + 1 = roll back to pod v (0: none)
#define s_vend s_ctl[1]       // verifier: the batch's committed count (-1: not yet)
#define s_verified s_ctl[2]   // verifier: pods verified (wave 0 decides at most SP_LAG ahead of it)
#define s_cut_at s_ctl[3]     // Reserve: the first pod whose cpuset the host selects (-1: none)
__shared__ int32_t s_decided, s_stop, s_parked, s_finish, s_err;
__shared__ int32_t s_werr;        // a verify / Reserve / re-scoring wave's bounded wait expired (its site code)
__shared__ int32_t s_jq_head[SP_NRES], s_jq_tail[SP_NRES];
__shared__ int32_t s_rb_at;       // the last rollback's pod (where the parked waves resume)
__shared__ int32_t s_end_at;      // wave 0: decisions end before this pod (B: every pod)
__shared__ int32_t s_vcut;        // verifier: a host cut ends the batch (with s_vend)
__shared__ int32_t s_committed, s_hostcut, s_nd, s_endwhy;
__shared__ int32_t s_snap;        // split: decisions whose slot table and batch-start scores the prep wave may read
__shared__ int32_t s_prep_done;   // split: pods the prep wave has recorded
__shared__ int32_t s_reprep;      // split: wave 0 -> prep wave: p + 1 = record pod p again over the exact state
__shared__ int32_t s_vlock, s_vwm;   // split, shared verification: the verifier's lock, its re-scored frontier

// (s_memtime is a scalar-memory instruction: reading its result waits for every LDS operation and scalar load in flight,
// so a stamp also closes the latency of the prefetches issued before it. HW_REG_SHADER_CYCLES reads 0 on gfx950.)
#define SPM(i)                                          \
  do {                                                  \
    if (ST) {                                           \
      const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
      st_acc[i] += t_ - st_last;                        \
      st_last = t_;                                     \
    }                                                   \
  } while (0)

__device__ __forceinline__ int32_t ld_acq(const int32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
__device__ __forceinline__ void st_rel(int32_t* p, int32_t v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
__device__ __forceinline__ uint64_t rfl64(uint64_t x) {   // a uniform 64-bit value into scalar registers
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}
typedef int32_t v4i32 __attribute__((ext_vector_type(4)));
// s_ctl as one snapshot: a 128-bit LDS read, then acquire (the words are written with release stores)
__device__ __forceinline__ v4i32 ld_ctl() {
  const v4i32 v = *reinterpret_cast<const volatile v4i32*>(s_ctl);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return v;
}


// ST: diagnostic build — per-role cycle sums (s_memtime) into a.stamps: 0 decide, 1 verify, 2 wave 0 waiting,
// 3 rollbacks, 4 rollback cycles, 5 Reserve busy, 6 Reserve waiting, 7 re-scoring busy, 8 re-scoring waiting,
// 9 decisions, 10 full-row decisions, 11 full-row cycles, 12 wave 0 total
template <bool ST, bool SPLIT>
__global__ void __launch_bounds__(SP_THREADS) commit_spec_kernel(CommitArgs a) {
  uint64_t st_acc[SP_NST] = {};
  uint64_t st_last = ST ? __builtin_amdgcn_s_memtime() : 0;
  const uint64_t st_t0 = st_last;
  const int B = a.npods;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const MirrorView& m = a.m;
  const bool numa_on = (a.pf.enabled & 0x30u) != 0;
  const bool multi = a.nranks > 1;   // merged levels of several shards; rows outside [own0, own1) have no S_own
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  // ---- LDS (fixed layout, SpecLds)
  extern __shared__ __align__(16) unsigned char cm[];
  SpecLds& L = *reinterpret_cast<SpecLds*>(cm);
  auto pods = [&](int i) -> PodVec& { return *reinterpret_cast<PodVec*>(L.pods_b + (size_t)i * POD_STRIDE); };
  Row* drows = L.drows;
  int16_t* dsc = L.dsc;   // [pod][slot], stride SB
  int16_t* dso = L.dso;
  CpuStateDev* cst = L.cst;
  DecRec* dec = L.dec;
  UndoRec* undo = L.undo;
  HintTable* tables = L.tables;
  int32_t* final_F = L.final_F;
  int32_t* done_ver = L.done_ver;   // slot: version whose re-scoring is complete
  int32_t* has_row = L.has_row;     // slot: row fetched into LDS
  int32_t* rescored = L.rescored;   // pod: Reserve + re-scoring complete
  int32_t* jobs_left = L.jobs_left; // pod: re-scoring jobs not done (-> done_ver)
  int32_t* jobs_all = L.jobs_all;   // pod: every job not done (-> rescored)
  int32_t* resv = L.resv;           // pod: its Reserve is applied (or FitError)
  int32_t* hkey = L.hkey;
  int16_t* hval = L.hval;
  Job* jobq = L.jobq;               // [Reserve wave][ring]

  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();   // the kernel's duration -> committed[4] (100 MHz ticks)
  if (a.prev && a.prev[1] != 1) {   // speculative pass behind a batch that left work for the host: no-op
    if (tid == 0) { a.committed[0] = -1; a.committed[1] = 0; a.committed[3] = 0; a.committed[4] = 0; }
    return;
  }
  if (a.xerr && a.xerr[0]) {   // the ranks' level blocks are not the same exchange (merge_levels): commit nothing
    if (tid == 0) { a.committed[0] = 0; a.committed[1] = 0; a.committed[2] = 0; a.committed[3] = COMMIT_ERR_XTAG; a.committed[4] = 0; }
    return;
  }
  for (int i = tid; i < B; i += SP_THREADS) {
    pods(i) = a.pods[i];
    done_ver[i] = -1;
    has_row[i] = 0;
    rescored[i] = 0;
    jobs_left[i] = 0;
    jobs_all[i] = 0;
    resv[i] = 0;
  }
  for (int i = tid; i < SP_HASH; i += SP_THREADS) { hkey[i] = -1; hval[i] = -1; }
  for (int i = tid; i < B; i += SP_THREADS) tiebreak_records(a.seed, a.seq[i], a.tb + (size_t)i * TB_N);
  if (tid == 0) {
    s_decided = 0; s_stop = 0; s_parked = 0; s_finish = 0; s_cut_at = -1; s_err = 0; s_werr = 0;
    for (int k = 0; k < SP_NRES; ++k) { s_jq_head[k] = 0; s_jq_tail[k] = 0; }
    s_verified = 0; s_rb_req = 0; s_end_at = B; s_vend = -1; s_vcut = 0;
    s_committed = 0; s_hostcut = 0; s_nd = 0;
    s_snap = 0; s_prep_done = 0; s_reprep = 0; s_vlock = 0; s_vwm = 0;
  }
  __syncthreads();


  // ---- shared by the deciding waves (wave 0; the prep wave of the split pipeline)
  // header of pod p (lanes 0..7: level j score / count) and the head of its level list (lane i: entry i)
  // (all LEVALL levels: the LevelHdr's first MAXLEV and the LevelExt's rest)
  auto load_hdr = [&](int p, Hdr& o) {
    const LevelHdr* h = hdr_ptr(a, 0, p);
    const LevelExt* x = reinterpret_cast<const LevelExt*>(a.xbase + (size_t)a.bmax * LCAP * 4 +
                                                          (size_t)a.bmax * sizeof(LevelHdr)) + p;
    o.nlev = x->nlev;
    o.feas = h->feasible;
    o.next = x->next;
    o.hs = lane < MAXLEV ? h->score[lane] : lane < LEVALL ? x->score[lane - MAXLEV] : -1;
    o.hc = lane < MAXLEV ? h->count[lane] : lane < LEVALL ? x->count[lane - MAXLEV] : 0;
    o.lh = list_ptr(a, 0, p)[lane];
    o.tbv = a.tb[(size_t)p * TB_N + (lane & (TB_N - 1))];
  };
  // tiebreak_position(a.seed, seq[p], T) from pod p's records (tbv, lane k: entry k)
  auto tb_pos = [&](int p, int32_t tbv, int64_t T) -> int64_t {
    const int32_t lim = __builtin_amdgcn_readlane(tbv, TB_N - 1);
    if (T > (int64_t)lim) return tiebreak_position(a.seed, a.seq[p], T);   // (past the records: rare)
    const int cnt = __popcll(__ballot(lane < TB_N - 1 && tbv != INT32_MAX && (int64_t)tbv <= T));
    return cnt ? (int64_t)__builtin_amdgcn_readlane(tbv, cnt - 1) : 1;
  };
  // selectHost of pod p over its levels and the dirty slots [0, nd) (slot s: node in lane s % 64 of dn0 / dn1, latest
  // decided version in pv0 / pv1): ready slots with their exact current score, pending ones left out. nh: where the
  // next pod's header loads go (issued once this pod's dirty-slot state is read); pre_dso: runs before the dso loads.
  // PREP (the split pipeline's prep wave): also the masks and the tie window the final decision needs (PrepRec).
  auto decide_core = [&](int p, const Hdr& h, Hdr& nh, bool want_next, auto&& pre_dso, int nd, uint32_t dn0, uint32_t dn1, int32_t pv0,
                         int32_t pv1, auto prep_tag, Dc& r) {
    constexpr bool PREP = decltype(prep_tag)::v;
    const int hs = h.hs, hc = h.hc, nlev = h.nlev, feas = h.feas, next = h.next;
    const uint32_t lh = h.lh;
    const int32_t tbv = h.tbv;
    auto each_node = [&](uint64_t m0, uint64_t m1, auto&& fn) {
      for (uint64_t b = m0; b; b &= b - 1) fn((uint32_t)__builtin_amdgcn_readlane((int)dn0, __builtin_ctzll(b)));
      for (uint64_t b = m1; b; b &= b - 1) fn((uint32_t)__builtin_amdgcn_readlane((int)dn1, __builtin_ctzll(b)));
    };
    r.action = 0;
    r.end_why = 0;
    r.winner = 0xffffffffu;
    r.ntw = 0;
    r.twv = 0xffffffffu;
    // dirty slots: ready (exact current score) or pending (left out)
    const int dv0 = lane < nd ? ld_acq(&done_ver[lane]) : -1;
    const int dv1 = lane + 64 < nd ? ld_acq(&done_ver[lane + 64]) : -1;
    const bool rdy0 = lane < nd && dv0 == pv0, rdy1 = lane + 64 < nd && dv1 == pv1;
    const uint64_t pend0 = __ballot(lane < nd && !rdy0), pend1 = __ballot(lane + 64 < nd && !rdy1);
    r.pend0 = pend0;
    r.pend1 = pend1;
    if ((a.dbg & 1u) && (pend0 | pend1)) {   // diagnostics: no speculation, wait for the pending rows
      r.action = 4;
      return;
    }
    SPM(28);   // dirty-slot state (versions, ballots)
    if (want_next && p + 1 < B) load_hdr(p + 1, nh);   // consumed by the next decision
    int sc0 = -1, so0 = -1, sc1 = -1, so1 = -1;
    pre_dso();
    if (lane < nd) { so0 = dso[p * SB + lane]; if (rdy0) sc0 = dsc[p * SB + lane]; }
    if (lane + 64 < nd) { so1 = dso[p * SB + 64 + lane]; if (rdy1) sc1 = dsc[p * SB + 64 + lane]; }
    SPM(29);   // next header's loads issued, pending fresh slot stored, dirty scores loaded
    uint64_t unk0 = 0, unk1 = 0;
    if (multi) {
      // off-shard fresh rows whose batch-start job has not finished: a node in the list head has its listed level
      // as batch-start score (exact); any other is unknown, counted as clean and unlisted (checked at verification)
      const uint64_t u0 = __ballot(lane < nd && so0 == SO_UNKNOWN), u1 = __ballot(lane + 64 < nd && so1 == SO_UNKNOWN);
      if (u0 | u1) {
        const int incl = wave_incl_scan(lane < nlev ? hc : 0);   // list end of level `lane`
        const int listed = __builtin_amdgcn_readlane(incl, 63);
        for (int pass = 0; pass < 2; ++pass)
          for (uint64_t bb = pass ? u1 : u0; bb; bb &= bb - 1) {
            const int s = __builtin_ctzll(bb);
            const uint32_t nn = (uint32_t)__builtin_amdgcn_readlane((int)(pass ? dn1 : dn0), s);
            const uint64_t f = __ballot(lane < listed && lh == nn);
            int sv = SO_UNLISTED;
            if (f) {
              const int e = __builtin_ctzll(f);
              sv = __builtin_amdgcn_readlane(hs, __popcll(__ballot(lane < nlev && incl <= e)));
            } else if (pass) {
              unk1 |= 1ull << s;
            } else {
              unk0 |= 1ull << s;
            }
            if (lane == s) { if (pass) so1 = sv; else so0 = sv; }
          }
      }
    }
    r.unk0 = unk0;
    r.unk1 = unk1;
    // action 0 commit, 1 FitError, 2 stop deciding before p, 3 full-row resolution (wave 0)
    int action = 0;
    uint32_t winner = 0xffffffffu;
    int M = -1, F = 0;
    int64_t T = 0, jp = 0;
    bool slowpath = p == 0 && a.forced_node >= 0;
    // the highest listed level that still holds a clean node: listed count minus the dirty rows listed there (their
    // batch-start score), from the top (usually the first level)
    int ctop = 0, Mclean = -1;
    for (int j = 0; j < nlev; ++j) {
      const int sj = __builtin_amdgcn_readlane(hs, j), cj = __builtin_amdgcn_readlane(hc, j);
      const int dj = __popcll(__ballot(so0 == sj)) + __popcll(__ballot(so1 == sj));
      if (cj > dj) { ctop = cj - dj; Mclean = sj; break; }
    }
    const int Md = wave_max(max(sc0, sc1));
    const int Fd = wave_sum((sc0 >= 0) - (so0 >= 0) + (sc1 >= 0) - (so1 >= 0));
    M = max(Mclean, Md);
    F = Fd + feas;
    SPM(18);   // decide: dirty-slot state, level scan
    if (slowpath) {
      M = a.forced_score;
      F = a.forced_feasible;
      T = a.forced_ties;
      winner = (uint32_t)a.forced_node;
    } else if (M < 0 && next < 0) {
      action = 1;   // every feasible node is listed, none clean, no dirty row feasible: FitError
    } else if (M <= next) {
      action = a.S != nullptr ? 3 : 2;
      if (action == 2) r.end_why = 3;
      if (ST) st_acc[M < 0 ? 13 : 14] += 1;
    } else if (M < 0) {
      action = 1;
    } else {
      const bool nw0 = sc0 == M, nw1 = sc1 == M;
      // clean listed ties: only at the top clean level (a higher M is a dirty row's: every listed node there is dirty)
      T = (int64_t)(M == Mclean ? ctop : 0) + __popcll(__ballot(nw0)) + __popcll(__ballot(nw1));
      jp = tb_pos(p, tbv, T);
      if (ST && !PREP && !SPLIT && p > 0 && !(dec[p - 1].flags & SP_FITERR)) {
        // diagnostics: a decision made before pod p-1's landing was known (its row as it stood) vs this one
        const DecRec& pd = dec[p - 1];
        const int sl = pd.slot;
        const int ov = (pd.flags & SP_FRESH) ? __builtin_amdgcn_readlane(sl < 64 ? so0 : so1, sl & 63)
                                              : (int)dsc[p * SB + sl];
        st_acc[47] += 1;
        st_acc[48] += ov > M ? 1 : 0;
        st_acc[49] += ov == M ? 1 : 0;
        st_acc[50] += (ov == M && tb_pos(p, tbv, T + 1) != jp) ? 1 : 0;
      }
      SPM(30);   // winner: ties, tie-break position
      // level M's segment of the list: offset = listed nodes above it, len = listed nodes at it (0: not listed)
      const uint64_t atm = __ballot(lane < nlev && hs == M);
      const int jm = atm ? __builtin_ctzll(atm) : nlev;
      const int len = atm ? __builtin_amdgcn_readlane(hc, jm) : 0;
      const int off = wave_sum(lane < jm && lane < nlev ? hc : 0);
      const uint64_t new0 = __ballot(nw0), new1 = __ballot(nw1);
      const uint64_t old0 = __ballot(so0 == M && lane < nd), old1 = __ballot(so1 == M && lane + 64 < nd);
      const int nnew = __popcll(new0) + __popcll(new1), nold = __popcll(old0) + __popcll(old1);
      if (nnew == 0 && nold == 0) {
        // no dirty row at M (then level M is listed: M is its clean level): the jp-th listed node of level M
        const int e = off + (int)jp - 1;
        winner = e < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)lh, e) : list_ptr(a, 0, p)[e];
        if (PREP) {   // the ties after it: listed nodes e+1, e+2, ...
          const int nk = (int)min<int64_t>(SP_KW, T - jp + 1);
          const int ek = e + lane;
          const uint32_t fromh = (uint32_t)__shfl((int)lh, ek & 63);
          if (lane < nk) r.twv = ek < 64 ? fromh : list_ptr(a, 0, p)[ek];
          r.ntw = nk;
        }
        if (ST) { st_acc[24] += e >= 32 ? 1 : 0; st_acc[25] += e >= 64 ? 1 : 0; }
      } else if (nnew == 0 && nold <= 61 - (PREP ? SP_KW - 1 : 0)) {
        // only listed nodes at M, some of them dirty rows no longer at M ("old"; the common case): the jp-th of the
        // others in list order lies in the window [jp-2, jp-1+nold] of level M's segment (<= 64 entries, one per
        // lane); old nodes before the window are those with a lower node id (the segment is in node order)
        if (ST) { st_acc[36] += 1; st_acc[32] += nold; }
        const int lo = (int)max<int64_t>(0, jp - 2);
        const int hi = (int)min<int64_t>(len - 1, jp - 1 + nold + (PREP ? SP_KW - 1 : 0));
        const int W = hi - lo + 1;
        const int e = off + lo + lane;
        const uint32_t fromh = (uint32_t)__shfl((int)lh, e & 63);
        uint32_t x = 0xffffffffu;
        if (lane < W) x = e < 64 ? fromh : list_ptr(a, 0, p)[e];
        const uint32_t win0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 0);
        SPM(46);   // winner (old-nodes path): level segment, window of the list
        bool ow = false;
        int base_old = 0;
        each_node(old0, old1, [&](uint32_t n) {
          base_old += n < win0 ? 1 : 0;
          ow |= x == n;
        });
        const uint64_t bo = __ballot(lane < W && ow);
        const int older = base_old + __popcll(bo & lt_mask);
        const int64_t rk = (int64_t)(lo + lane - older + 1);   // the lane's rank among the ties
        const uint64_t hit = __ballot(lane < W && !ow && rk == jp);
        if (ST) { st_acc[24] += off + hi >= 32 ? 1 : 0; st_acc[25] += off + hi >= 64 ? 1 : 0; }
        if (!hit) { action = 2; r.end_why = 1; }
        else winner = (uint32_t)__builtin_amdgcn_readlane((int)x, __builtin_ctzll(hit));
        if (PREP && hit) {   // the ties ranked jp .. jp+SP_KW-1
          r.twv = winner;
          int k = 1;
          for (; k < SP_KW; ++k) {
            const uint64_t hk = __ballot(lane < W && !ow && rk == jp + k);
            if (!hk) break;
            const uint32_t xk = (uint32_t)__builtin_amdgcn_readlane((int)x, __builtin_ctzll(hk));
            if (lane == k) r.twv = xk;
          }
          r.ntw = k;
        }
      } else {
        if (ST) { st_acc[31] += 1; st_acc[32] += nold; st_acc[33] += nnew; }
        const int lo = (int)max<int64_t>(0, jp - 2 - nnew);
        const int hi = (int)min<int64_t>(len - 1, jp - 1 + nold);
        const int W = hi - lo + 1;
        if (ST) st_acc[34] += W > 0 ? W : 0;
        const uint32_t* L = list_ptr(a, 0, p);
        constexpr int WCH = (2 * MAX_BATCH + 2 + 63) / 64;
        uint32_t xw[WCH];
        bool ow[WCH];
        uint32_t cand = 0xffffffffu;
        int base_old = 0;
        if (len > 0) {
#pragma unroll
          for (int c = 0; c < WCH; ++c) {
            const int i = c * 64 + lane, e = off + lo + i;
            const uint32_t fromh = (uint32_t)__shfl((int)lh, e & 63);
            xw[c] = 0xffffffffu;
            if (c * 64 < W && i < W) xw[c] = e < 64 ? fromh : L[e];
          }
          if (ST) { st_acc[24] += off + hi >= 32 ? 1 : 0; st_acc[25] += off + hi >= 64 ? 1 : 0; }
          const uint32_t win0 = (uint32_t)__builtin_amdgcn_readlane((int)xw[0], 0);
#pragma unroll
          for (int c = 0; c < WCH; ++c) ow[c] = false;
          each_node(old0, old1, [&](uint32_t n) {
            base_old += n < win0 ? 1 : 0;
#pragma unroll
            for (int c = 0; c < WCH; ++c) ow[c] |= xw[c] == n;
          });
          int running = base_old;
#pragma unroll
          for (int c = 0; c < WCH; ++c) {
            if (c * 64 >= W) break;
            const int i = c * 64 + lane;
            const bool valid = i < W;
            const uint64_t bo = __ballot(valid && ow[c]);
            const int older = running + __popcll(bo & lt_mask);
            int newer = 0;
            each_node(new0, new1, [&](uint32_t n) { newer += n < xw[c] ? 1 : 0; });
            if (valid && !ow[c] && (int64_t)(lo + i - older + newer + 1) == jp) cand = xw[c];
            running += __popcll(bo);
          }
        }
        each_node(new0, new1, [&](uint32_t n) {
          int u = 0;
          each_node(new0, new1, [&](uint32_t n2) { u += n2 < n ? 1 : 0; });
          int64_t ltn = -1;
          int older = 0;
          if (len == 0) {
            ltn = 0;
          } else {
            int pp = 0;
#pragma unroll
            for (int c = 0; c < WCH; ++c) {
              if (c * 64 >= W) break;
              const bool valid = c * 64 + lane < W;
              pp += __popcll(__ballot(valid && xw[c] < n));
              older += __popcll(__ballot(valid && ow[c] && xw[c] < n));
            }
            older += base_old;
            if (pp == 0) ltn = (lo == 0) ? 0 : -1;
            else if (pp == W) ltn = (hi == len - 1) ? len : -1;
            else ltn = lo + pp;
          }
          if (ltn >= 0 && ltn - older + u + 1 == jp) cand = n;
        });
        const uint64_t got = __ballot(cand != 0xffffffffu);
        if (!got) { action = 2; r.end_why = 1; }
        else winner = (uint32_t)__builtin_amdgcn_readlane((int)cand, __ffsll((long long)got) - 1);
        if (PREP && got) {   // the window is the winner alone: any tie excluded before it leaves p to wave 0
          r.twv = winner;
          r.ntw = 1;
        }
      }
    }
    SPM(19);   // decide: tie-break position, winner among listed + dirty ties
    r.action = action;
    r.winner = winner;
    r.M = M;
    r.F = F;
    r.T = T;
    r.jp = jp;
    r.slowpath = slowpath;
    r.Mclean = Mclean;
    r.Md = Md;
    r.Fd = Fd;
    r.sc0 = sc0;
    r.sc1 = sc1;
    r.so0 = so0;
    r.so1 = so1;
    if (PREP) {
      const bool tok = M >= 0 && action == 0;
      r.sf0 = (rdy0 ? SF_READY : 0) | (sc0 >= 0 ? SF_FEAS : 0) | (tok && sc0 == M ? SF_TIE : 0) |
              (lane < nd && !rdy0 ? SF_PEND : 0);
      r.sf1 = (rdy1 ? SF_READY : 0) | (sc1 >= 0 ? SF_FEAS : 0) | (tok && sc1 == M ? SF_TIE : 0) |
              (lane + 64 < nd && !rdy1 ? SF_PEND : 0);
    }
  };

  // node -> slot hash, needed only by the full-row resolution: rebuilt there when slots changed since (one lane per
  // slot; an LDS compare-and-swap claims a probe position, and a key only moves past occupied positions, so
  // linear-probe lookups find it)
  auto rebuild_hash = [&](int nd, uint32_t dn0, uint32_t dn1) {
    for (int i = lane; i < SP_HASH; i += 64) { hkey[i] = -1; hval[i] = -1; }
    WAVE_FENCE();
    for (int half = 0; half < 2; ++half) {
      bool todo = lane + 64 * half < nd;
      const uint32_t nn = half ? dn1 : dn0;
      uint32_t h = (nn * 2654435761u) & (SP_HASH - 1);
      while (todo) {
        if (atomicCAS(&hkey[h], -1, (int32_t)nn) == -1) {
          hval[h] = (int16_t)(lane + 64 * half);
          todo = false;
        } else {
          h = (h + 1) & (SP_HASH - 1);
        }
      }
      WAVE_FENCE();
    }
  };
  auto sp_hash_find = [&](uint32_t node) -> int {
    uint32_t h = (node * 2654435761u) & (SP_HASH - 1);
    for (int probe = 0; probe < SP_HASH; ++probe) {
      const int kk = hkey[h];
      if (kk == (int)node) return hval[h];
      if (kk < 0) return -1;
      h = (h + 1) & (SP_HASH - 1);
    }
    return -1;
  };
  // ------------------------------------------------ exact resolution of pod p from its whole score row
  // batch-start S[p][*] for clean nodes, the current score for ready dirty rows, pending rows left out (verified
  // later like any decision)
  auto full_row_resolve = [&](int p, int32_t tbv, Dc& r, int nd, uint32_t dn0, uint32_t dn1, bool& hash_ok) {
    if (!hash_ok) {
      rebuild_hash(nd, dn0, dn1);
      hash_ok = true;
    }
    auto each_node = [&](uint64_t m0, uint64_t m1, auto&& fn) {
      for (uint64_t b = m0; b; b &= b - 1) fn((uint32_t)__builtin_amdgcn_readlane((int)dn0, __builtin_ctzll(b)));
      for (uint64_t b = m1; b; b &= b - 1) fn((uint32_t)__builtin_amdgcn_readlane((int)dn1, __builtin_ctzll(b)));
    };
    const int sc0 = r.sc0, sc1 = r.sc1, so0 = r.so0, so1 = r.so1, Md = r.Md, Fd = r.Fd;
    const int16_t* row = a.S + (size_t)p * a.ld;
    const uint32_t len = a.own1 - a.own0;
    constexpr int VB = 8;
    auto load_blk = [&](uint32_t i0, int16_t (&x)[8]) {
      if (i0 + 8 <= len) {
        const uint4 vv = *reinterpret_cast<const uint4*>(row + i0);
        const uint32_t w[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = (int16_t)(w[k >> 1] >> (16 * (k & 1)));
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = i0 + k < len ? row[i0 + k] : (int16_t)-1;
      }
    };
    int lmax = -1, lcnt = 0, lfeas = 0;
    for (uint32_t b0 = 0; b0 < len; b0 += 512u * VB) {
      int16_t x[VB][8];
#pragma unroll
      for (int u = 0; u < VB; ++u) load_blk(b0 + 512u * u + 8u * lane, x[u]);
#pragma unroll
      for (int u = 0; u < VB; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int xv = x[u][k];
          lfeas += xv >= 0 ? 1 : 0;
          lcnt = xv > lmax ? 1 : lcnt + (xv == lmax ? 1 : 0);
          lmax = xv > lmax ? xv : lmax;
        }
    }
    r.F = wave_sum(lfeas) + Fd;
    int Mc = wave_max(lmax);
    int64_t Tc = Mc >= 0 ? (int64_t)wave_sum(lmax == Mc ? lcnt : 0) - __popcll(__ballot(lane < nd && so0 == Mc)) -
                               __popcll(__ballot(lane + 64 < nd && so1 == Mc))
                         : 0;
    if (Mc >= 0 && Tc <= 0) {
      lmax = -1;
      lcnt = 0;
      for (uint32_t b0 = 0; b0 < len; b0 += 512u * VB) {
        int16_t x[VB][8];
#pragma unroll
        for (int u = 0; u < VB; ++u) load_blk(b0 + 512u * u + 8u * lane, x[u]);
#pragma unroll
        for (int u = 0; u < VB; ++u)
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int xv = x[u][k];
            if (xv >= 0 && xv >= lmax && sp_hash_find(a.own0 + b0 + 512u * u + 8u * lane + k) < 0) {
              lcnt = xv > lmax ? 1 : lcnt + 1;
              lmax = xv;
            }
          }
      }
      Mc = wave_max(lmax);
      Tc = Mc >= 0 ? (int64_t)wave_sum(lmax == Mc ? lcnt : 0) : 0;
    }
    const int M = max(Mc, Md);
    r.M = M;
    if (M < 0) {
      r.action = 1;
      return;
    }
    const uint64_t new0 = __ballot(sc0 == M), new1 = __ballot(sc1 == M);
    const uint64_t old0 = __ballot(lane < nd && so0 == M), old1 = __ballot(lane + 64 < nd && so1 == M);
    const int64_t T = (Mc == M ? Tc : 0) + __popcll(new0) + __popcll(new1);
    r.T = T;
    const int64_t jp = tb_pos(p, tbv, T);
    int64_t run = 0;
    int64_t found = -1;
    for (uint32_t b0 = 0; b0 < len && found == -1; b0 += 512u * VB) {
      int16_t x[VB][8];
#pragma unroll
      for (int u = 0; u < VB; ++u) load_blk(b0 + 512u * u + 8u * lane, x[u]);
#pragma unroll
      for (int u = 0; u < VB; ++u) {
        const uint32_t i0 = b0 + 512u * u;
        uint32_t fl = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) fl |= (x[u][k] == M ? 1u : 0u) << k;
        const bool in0 = dn0 - a.own0 - i0 < 512u, in1 = dn1 - a.own0 - i0 < 512u;
        const uint64_t bn0 = new0 & __ballot(in0), bn1 = new1 & __ballot(in1);
        const uint64_t bo0 = old0 & __ballot(in0), bo1 = old1 & __ballot(in1);
        const int tot = wave_sum(__popc(fl)) + __popcll(bn0) + __popcll(bn1) - __popcll(bo0) - __popcll(bo1);
        if (found == -1 && run + tot >= jp) {
          each_node(bo0, bo1, [&](uint32_t nn) {
            const uint32_t o = nn - a.own0 - i0;
            if ((uint32_t)lane == (o >> 3)) fl &= ~(1u << (o & 7u));
          });
          each_node(bn0, bn1, [&](uint32_t nn) {
            const uint32_t o = nn - a.own0 - i0;
            if ((uint32_t)lane == (o >> 3)) fl |= 1u << (o & 7u);
          });
          const int c = __popc(fl);
          const int incl = wave_incl_scan(c);
          int64_t need = jp - (run + incl - c);
          int64_t f = -1;
          if (need >= 1 && need <= c) {
            uint32_t bits = fl;
            while (--need) bits &= bits - 1;
            f = (int64_t)(a.own0 + i0 + 8u * lane + (uint32_t)__builtin_ctz(bits));
          }
          const uint64_t gg = __ballot(f >= 0);
          found = gg ? (int64_t)__builtin_amdgcn_readlane((int)f, __ffsll((long long)gg) - 1) : -2;
        }
        run += tot;
      }
    }
    if (found < 0) {
      r.action = 2;
      r.end_why = 2;
      const int osl = old0 ? __builtin_ctzll(old0) : old1 ? 64 + __builtin_ctzll(old1) : -1;
      const uint32_t onode = osl < 0 ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)(osl < 64 ? dn0 : dn1), osl & 63);
      const int ohash = osl < 0 ? -9 : sp_hash_find(onode);
      const int osv = osl < 0 ? -9 : (int)a.S[(size_t)p * a.ld + (onode - a.own0)];
      const int odso = osl < 0 ? -9 : (int)dso[p * SB + osl];
      if (lane == 0)   // diagnostics (GS_DEBUG_CUTS): the inconsistent tie count
        a.out[p] = PlacementDev{-7, (uint32_t)run, (int64_t)M | ((int64_t)Mc << 20) | ((int64_t)Md << 40), (uint32_t)T,
                                (uint32_t)Tc, (uint32_t)(__popcll(new0) + __popcll(new1)),
                                (uint32_t)(__popcll(old0) + __popcll(old1)), {(int64_t)jp, (int64_t)nd, (int64_t)__popcll(r.pend0), 0}, {0, 0, 0, 0},
                                {(uint64_t)osl, (uint64_t)onode, (uint64_t)(int64_t)ohash,
                                 (uint64_t)(((int64_t)osv << 32) | (uint32_t)odso)}};
    } else {
      r.action = 0;
      r.winner = (uint32_t)found;
    }
    r.slowpath = true;
  };
  // split pipeline, shared verification (dbg bit 17): the decided pods verified in order by whichever wave holds the
  // lock — the re-scoring and Reserve waves when they complete a pod's re-scoring, wave 0 while it waits. Same rule
  // as the verify wave: pod v stands iff every row pending at its decision now scores below its maximum for it (its
  // feasible ones join the Feasible count); a miss asks wave 0 to roll back to v (s_rb_req).
  const bool vshare = SPLIT && ((a.dbg >> 17) & 1u);
  // (dbg bit 19, with 17: the prep wave verifies while it waits for the ring, the re-scoring / Reserve waves do not)
  const bool vprep = vshare && ((a.dbg >> 19) & 1u);
  // pods the prep wave may work ahead of wave 0's decisions: 1 + 1 (GS_SPEC_AHEAD=2, dbg bit 18: + 2)
  const int prep_ahead = ((a.dbg >> 18) & 1u) ? SP_PREPQ : SP_PREPQ - 1;
  auto verify_try = [&]() {
    int got = 0;
    if (lane == 0) {
      int expect = 0;
      got = __atomic_compare_exchange_n(&s_vlock, &expect, 1, false, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED) ? 1 : 0;
    }
    if (!__builtin_amdgcn_readfirstlane(got)) return;
    if (!ld_acq(&s_rb_req) && !ld_acq(&s_stop)) {
      int v = ld_acq(&s_verified), wm = ld_acq(&s_vwm);
      const int qd = ld_acq(&s_decided);
      while (wm < qd && ld_acq(&rescored[wm])) ++wm;
      const int cut_v = ld_acq(&s_cut_at);   // (after the frontier: a cut is published before its pod is re-scored)
      while (v < qd && v <= wm) {
        if (cut_v >= 0 && v > cut_v) break;
        const DecRec& d = dec[v];
        const uint64_t dp0 = d.pend0, dp1 = d.pend1;
        const int dM = d.M;
        int mis = 0, fadd = 0;
        if ((dp0 >> lane) & 1ull) {
          const int sc = dsc[v * SB + lane];
          mis |= sc >= 0 && sc >= dM;
          fadd += sc >= 0;
        }
        if ((dp1 >> lane) & 1ull) {
          const int sc = dsc[v * SB + 64 + lane];
          mis |= sc >= 0 && sc >= dM;
          fadd += sc >= 0;
        }
        if (__ballot(mis)) {
          if (lane == 0) st_rel(&s_rb_req, v + 1);
          break;
        }
        const int F = d.F + wave_sum(fadd);
        if (lane == 0) final_F[v] = F;
        ++v;
      }
      if (lane == 0) {
        s_vwm = wm;
        st_rel(&s_verified, v);
      }
    }
    WAVE_FENCE();
    if (lane == 0) st_rel(&s_vlock, 0);
  };

  if (wv == 0) {
    // ==================================================== decide ====================================================
    __builtin_amdgcn_s_setprio(3);
    // decisions ahead of the verifier: SP_LAG (the undo log's depth), or fewer (GS_SPEC_LAG, experiments)
    const int lag = ((a.dbg >> 12) & 15u) ? (int)min((a.dbg >> 12) & 15u, (uint32_t)SP_LAG) : SP_LAG;
    uint32_t dn0 = 0xffffffffu, dn1 = 0xffffffffu;   // slot s's node in lane s % 64 of dn0 / dn1
    int32_t pv0 = -1, pv1 = -1;                      // slot s's latest decided version (pod index)
    int nd = 0, q = 0, end_at = B, end_why = 0;
    int committed = 0;
    bool host_cut = false, err = false;
    int err_code = 0;   // which bounded wait expired (reported in committed[3])
    bool hash_ok = true;   // the node -> slot hash matches the slots (full-row resolution)
    // a fresh slot's batch-start scores for the later pods (S_own column loads), issued when the slot is created and
    // stored into dso by the next decision (the loads' latency hides behind the verification in between)
    int ps_slot = -1, ps_p = 0;
    int16_t ps_v0 = 0, ps_v1 = 0;
    auto flush_fresh = [&]() {
      if (ps_slot < 0) return;
      const int q0 = ps_p + 1 + lane, q1 = q0 + 64;
      if (q0 < B) dso[q0 * SB + ps_slot] = ps_v0;
      if (q1 < B) dso[q1 * SB + ps_slot] = ps_v1;
      ps_slot = -1;
    };
    Hdr nh{-1, 0, 0, 0, -1, 0xffffffffu, 1};
    if (!SPLIT) load_hdr(0, nh);
    uint32_t spins = 0;
    int ver = 0, wm = 0;   // split pipeline: pods verified here, the re-scored frontier
    // ------------------------------------------------ roll back to pod v
    auto rollback = [&](int v) -> bool {
      if (ST) {
        st_acc[43] += (dec[v].flags & SP_PRED_GE) ? 1 : 0;
        st_acc[45] += (dec[v].flags & SP_PRED_GT) ? 1 : 0;
      }
      // park the other waves, undo the Reserves of pods >= v (newest first: the two Reserve waves finish pods out of
      // order, so by their flags), restore the slot versions
      st_rel(&s_stop, 1);
      spins = 0;
      while (ld_acq(&s_parked) < SP_WAVES - 1) {
        if (++spins > SP_SPIN_LIMIT) { err = true; err_code = 1; return false; }
        sp_sleep();
      }
      SPM(37);   // rollback: parking the other waves
      if (ST) st_acc[41] += q - v;
      for (int qq = q - 1; qq >= v; --qq) {
        if (!resv[qq] || (dec[qq].flags & SP_FITERR)) continue;
        const UndoRec& u = undo[qq % SP_LAG];
        const int sl = u.slot;
        const uint64_t* src = reinterpret_cast<const uint64_t*>(&u.row);
        uint64_t* dst = reinterpret_cast<uint64_t*>(&drows[sl]);
        for (int i = lane; i < (int)(sizeof(Row) / 8); i += 64) dst[i] = src[i];
        const uint64_t* s2 = reinterpret_cast<const uint64_t*>(&u.cs);
        uint64_t* d2 = reinterpret_cast<uint64_t*>(&cst[sl]);
        for (int i = lane; i < (int)(sizeof(CpuStateDev) / 8); i += 64) d2[i] = s2[i];
        WAVE_FENCE();
      }
      // versions of the slots that survive, newest undone landing first
      uint64_t redo0 = 0, redo1 = 0;   // surviving slots whose row was restored: re-score them for pods >= v
      for (int qq = q - 1; qq >= v; --qq) {
        const DecRec& e = dec[qq];
        if ((e.flags & (SP_FITERR | SP_FRESH)) || e.slot >= dec[v].nd_before) continue;
        const int sl = e.slot;
        if (lane == (sl & 63)) { if (sl < 64) pv0 = e.prev_pend; else pv1 = e.prev_pend; }
        if (resv[qq]) { if (sl < 64) redo0 |= 1ull << sl; else redo1 |= 1ull << (sl - 64); }
      }
      const int ndv = dec[v].nd_before;
      ps_slot = -1;   // a pending fresh slot is the last decision's: >= ndv, undone
      if (lane >= ndv) { dn0 = 0xffffffffu; pv0 = -1; }
      if (lane + 64 >= ndv) { dn1 = 0xffffffffu; pv1 = -1; }
      for (int s = ndv + lane; s < nd; s += 64) { has_row[s] = 0; done_ver[s] = -1; }
      nd = ndv;
      hash_ok = false;   // rebuilt by the next full-row resolution that needs it
      SPM(38);   // rollback: undo log, slot versions
      if (ST) st_acc[40] += __popcll(redo0) + __popcll(redo1);
      // re-score the restored rows for pods v.. (their dsc entries after the undone landing are stale)
      for (int pass = 0; pass < 2; ++pass) {
        for (uint64_t bb = pass ? redo1 : redo0; bb; bb &= bb - 1) {
          const int sl = (pass ? 64 : 0) + __builtin_ctzll(bb);
          const Row rr = drows[sl];
          // (the re-scoring waves are parked: wave 0 borrows the first one's hint table)
          if (numa_on && ((rr.nr.nflags >> NF_POLICY_SHIFT) & 3u)) hint_table_fill(tables[0], rr.nr, zone_avail(rr.nr), lane);
          WAVE_FENCE();
          for (int q2 = v + lane; q2 < B; q2 += 64) dsc[q2 * SB + sl] = (int16_t)row_score(rr, pods(q2), a.pf, m, &tables[0]);
          WAVE_FENCE();
        }
      }
      SPM(39);   // rollback: re-scoring the restored rows
      const int32_t myv0 = pv0, myv1 = pv1;
      if (lane < nd) done_ver[lane] = myv0;
      if (lane + 64 < nd) done_ver[lane + 64] = myv1;
      if (SPLIT) {   // the slot table the prep wave snapshots
        if (lane < nd) L.slot_pv[lane] = myv0;
        if (lane + 64 < nd) L.slot_pv[lane + 64] = myv1;
      }
      for (int qq = v + lane; qq < B; qq += 64) {
        rescored[qq] = 0;
        jobs_left[qq] = 0;
        jobs_all[qq] = 0;
        resv[qq] = 0;
      }
      if (lane == 0) {
        for (int k = 0; k < SP_NRES; ++k) { s_jq_head[k] = 0; s_jq_tail[k] = 0; }
        if (s_cut_at >= v) s_cut_at = -1;   // a cut before v stands (its pod is not undone)
        s_decided = v;
        s_verified = v;
        s_rb_at = v;
        s_end_at = B;
        s_snap = v;
        s_prep_done = v;
        s_reprep = 0;
        s_vwm = v;
        s_parked = 0;
        s_rb_req = 0;
      }
      WAVE_FENCE();
      q = v;
      ver = v;
      wm = v;
      end_at = B;
      end_why = 0;
      if (lane == 0) st_rel(&s_stop, 0);
      if (!SPLIT) {
        nh.hs = -1;   // reload pod v's header
        load_hdr(v, nh);
      }
      if (ST) st_acc[3] += 1;
      SPM(4);
      return true;
    };
    // ------------------------------------------------ record decision p, claim / version the winner's slot
    auto record = [&](int p, const Dc& r) {
      const int action = r.action;
      const uint32_t winner = r.winner;
      DecRec d{};
      d.winner = action == 1 ? -1 : (int32_t)winner;
      d.M = action == 1 ? -1 : r.M;
      d.T = (int32_t)r.T;
      d.F = r.F;
      d.nd_before = nd;
      d.pend0 = r.pend0;
      d.pend1 = r.pend1;
      d.unk0 = r.unk0;
      d.unk1 = r.unk1;
      d.flags = (action == 1 ? SP_FITERR : 0u) | (r.slowpath ? SP_SLOW : 0u);
      if (ST && !SPLIT && action == 0 && (r.pend0 | r.pend1)) {
        // would a rule "wait when a pending row scored >= M (> M) for p before its landing" have foreseen the rollbacks?
        int o0 = -1, o1 = -1;
        if ((r.pend0 >> lane) & 1ull) o0 = dec[pv0].prev_pend < 0 ? r.so0 : (int)dsc[p * SB + lane];
        if ((r.pend1 >> lane) & 1ull) o1 = dec[pv1].prev_pend < 0 ? r.so1 : (int)dsc[p * SB + 64 + lane];
        const int om = wave_max(max(o0, o1));
        if (om >= r.M) { d.flags |= SP_PRED_GE; st_acc[42] += 1; }
        if (om > r.M) { d.flags |= SP_PRED_GT; st_acc[44] += 1; }
      }
      d.slot = -1;
      d.prev_pend = -1;
      if (action == 0) {
        const uint64_t hit0 = __ballot(dn0 == winner), hit1 = __ballot(dn1 == winner);
        int slot = hit0 ? __builtin_ctzll(hit0) : hit1 ? 64 + __builtin_ctzll(hit1) : -1;
        if (slot < 0) {   // fresh row: a new slot, its batch-start scores for the later pods
          slot = nd;
          d.flags |= SP_FRESH;
          if (lane == (nd & 63)) { if (nd < 64) { dn0 = winner; pv0 = p; } else { dn1 = winner; pv1 = p; } }
          const int q0 = p + 1 + lane, q1 = q0 + 64;
          if (winner - a.own0 < a.own1 - a.own0) {
            // both loads issued unconditionally (rows clamped into the batch; flush_fresh stores only q < B): no exec-mask
            // branch between them, so neither waits for the other, nor for the next header's loads in flight
            const int16_t* col = a.S_own + (winner - a.own0);
            ps_v0 = col[(size_t)min(q0, B - 1) * a.ld];
            ps_v1 = col[(size_t)min(q1, B - 1) * a.ld];
            ps_slot = slot;
            ps_p = p;
          } else {   // another shard's row: unknown until the Reserve wave's batch-start job has evaluated it
            d.flags |= SP_OFFSHARD;
            if (q0 < B) dso[q0 * SB + slot] = SO_UNKNOWN;
            if (q1 < B) dso[q1 * SB + slot] = SO_UNKNOWN;
          }
          if (lane == 0) done_ver[slot] = -1;
          hash_ok = false;
          ++nd;
          SPM(20);   // decide: fresh slot's batch-start scores (S_own loads)
        } else {          // a ready dirty row lands another pod: pending again
          const int32_t prevv = slot < 64 ? __builtin_amdgcn_readlane(pv0, slot) : __builtin_amdgcn_readlane(pv1, slot - 64);
          d.prev_pend = prevv;
          if (lane == (slot & 63)) { if (slot < 64) pv0 = p; else pv1 = p; }
        }
        d.slot = slot;
        if (SPLIT && lane == 0) {   // the slot table the prep wave snapshots
          L.slot_node[slot] = (int32_t)winner;
          L.slot_pv[slot] = p;
        }
      }
      if (lane == 0) dec[p] = d;
      WAVE_FENCE();
      if (lane == 0) st_rel(&s_decided, p + 1);
      if (ST) st_acc[9] += 1;
      SPM(0);
    };
    // ------------------------------------------------ split pipeline: verification of the decided pods, in order
    // pod v stands iff every row pending at its decision now scores below its maximum for it; the rows it excluded
    // that are feasible join its Feasible count (same rule as the verify wave of the unsplit pipeline). 0: nothing
    // more now, 1: roll back to `ver`, 2: the batch ends at `committed`.
    auto verify_step = [&](int cut_at) -> int {
      while (wm < q && ld_acq(&rescored[wm])) ++wm;
      while (ver < q && ver <= wm) {
        if (cut_at >= 0 && ver > cut_at) break;
        const DecRec& d = dec[ver];
        const uint64_t dp0 = d.pend0, dp1 = d.pend1;
        const int dM = d.M;
        int mis = 0, fadd = 0;
        if ((dp0 >> lane) & 1ull) {
          const int sc = dsc[ver * SB + lane];
          mis |= sc >= 0 && sc >= dM;
          fadd += sc >= 0;
        }
        if ((dp1 >> lane) & 1ull) {
          const int sc = dsc[ver * SB + 64 + lane];
          mis |= sc >= 0 && sc >= dM;
          fadd += sc >= 0;
        }
        if (__ballot(mis)) return 1;
        const int F = d.F + wave_sum(fadd);
        if (lane == 0) final_F[ver] = F;
        ++ver;
      }
      // a Reserve that needs the host's cpuset selection ends the batch right after its pod
      if (cut_at >= 0 && ver > cut_at) { committed = cut_at + 1; host_cut = true; return 2; }
      if (ver == end_at) { committed = ver; return 2; }   // every pod before the end of the decisions is verified
      return 0;
    };
    // ------------------------------------------------ split pipeline: the final decision of pod p from its PrepRec
    // The prep wave decided p over a snapshot of the decisions before rec.q_s; the decisions [q_s, p) landed after it.
    // Each such landing makes its slot pending: a slot the snapshot held as ready loses its exact score (a tie at M is
    // excluded, its feasibility leaves F); a slot created after the snapshot was a clean node to the prep wave (a
    // clean tie at M is excluded, its batch-start feasibility leaves F). M stands (exclusions only lower the field); the
    // tie-break position stands while T' >= jp (records are a prefix property); the winner is the jp-th of the
    // remaining ties, found in the window of ties the prep wave recorded. false: p needs a full decision here.
    auto apply_late = [&](int p, Dc& r) -> bool {
      const PrepRec& rec = L.prq[p % SP_PREPQ];
      // the record (five 16-byte words, uniform), the late decisions (lane i: decision q_s + i) and the snapshot's slot
      // flags (lane: slot lane / lane + 64), read together
      typedef int32_t i4 __attribute__((ext_vector_type(4)));
      const i4 h0 = reinterpret_cast<const i4*>(&rec)[0], h1 = reinterpret_cast<const i4*>(&rec)[1];
      const i4 h2 = reinterpret_cast<const i4*>(&rec)[2], h3 = reinterpret_cast<const i4*>(&rec)[3];
      const uint32_t twv = lane < SP_KW ? rec.tw[lane] : 0xffffffffu;
      const int pod = __builtin_amdgcn_readfirstlane(h0.x), qs = __builtin_amdgcn_readfirstlane(h0.y);
      const int nds = __builtin_amdgcn_readfirstlane(h0.z), action = __builtin_amdgcn_readfirstlane(h0.w);
      const int sfa = lane < nds ? rec.sf[lane] : 0, sfb = lane + 64 < nds ? rec.sf[lane + 64] : 0;
      const int nl = p - qs;
      int s = -1;
      uint32_t w = 0, fl = SP_FITERR;
      if (lane < nl) {
        const DecRec& e = dec[qs + lane];
        fl = e.flags;
        s = e.slot;
        w = (uint32_t)e.winner;
      }
      if (pod != p || nl > 64 || action > 2 || (action == 2 && nl != 0)) return false;
      SPM(52);   // split: the record, the late decisions
      if (action == 2) {   // stop deciding before p (an exact record)
        r.action = 2;
        r.end_why = __builtin_amdgcn_readfirstlane(h2.x);
        return true;
      }
      const int M = __builtin_amdgcn_readfirstlane(h1.x), Mclean = __builtin_amdgcn_readfirstlane(h1.y);
      const int F0 = __builtin_amdgcn_readfirstlane(h1.z), ntw = __builtin_amdgcn_readfirstlane(h1.w);
      const bool val = lane < nl && !(fl & SP_FITERR);
      // a slot landed on twice after the snapshot counts once; lt0 / lt1: slot lane / lane + 64 landed on since
      bool dup = false, lt0 = false, lt1 = false;
      for (int j = 0; j < nl; ++j) {
        const int sj = __builtin_amdgcn_readlane(s, j);
        dup |= lane > j && s == sj;
        lt0 |= lane == sj;
        lt1 |= lane + 64 == sj;
      }
      const bool use = val && !dup;
      const bool in_snap = s < nds;
      int sfv = 0, so = -1;
      if (use) {
        if (in_snap) sfv = rec.sf[s];
        else so = dso[p * SB + s];
      }
      // a slot the snapshot held ready loses its exact score (tie / feasible); one created after it was a clean node
      const bool fdec = use && (in_snap ? (sfv & SF_FEAS) != 0 : so >= 0);
      const bool tie = use && action == 0 && (in_snap ? (sfv & SF_TIE) != 0 : so == M && M == Mclean);
      // (a clean node above M cannot be: the prep wave's M is at least its clean level)
      if (__ballot(use && !in_snap && so > M && action == 0)) return false;
      int F = F0 - __popcll(__ballot(fdec));
      const int ne = __popcll(__ballot(tie));
      SPM(53);   // split: the late slots' exclusions
      // rows pending at the snapshot, not landed on since, whose re-scoring is complete now: their exact score for p
      // settles them here (one at or above M: p is recorded again over the exact state, instead of a rollback later)
      bool chk0 = (sfa & SF_PEND) && !lt0, chk1 = (sfb & SF_PEND) && !lt1;
      if (chk0) chk0 = ld_acq(&done_ver[lane]) == pv0;
      if (chk1) chk1 = ld_acq(&done_ver[lane + 64]) == pv1;
      int sc0 = -1, sc1 = -1;
      if (chk0) sc0 = dsc[p * SB + lane];
      if (chk1) sc1 = dsc[p * SB + 64 + lane];
      if (__ballot((sc0 >= 0 && sc0 >= M) || (sc1 >= 0 && sc1 >= M))) return false;
      F += wave_sum((sc0 >= 0 ? 1 : 0) + (sc1 >= 0 ? 1 : 0));
      SPM(54);   // split: rows settled early
      r.action = action;
      r.M = M;
      r.F = F;
      r.T = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(h2.w) << 32) |
                      (uint32_t)__builtin_amdgcn_readfirstlane(h2.z));
      r.pend0 = __ballot((((sfa & SF_PEND) != 0) || lt0) && !chk0);
      r.pend1 = __ballot((((sfb & SF_PEND) != 0) || lt1) && !chk1);
      r.unk0 = 0;
      r.unk1 = 0;
      r.slowpath = __builtin_amdgcn_readfirstlane(h2.y) != 0;
      r.end_why = 0;
      r.winner = 0xffffffffu;
      if (ST) { st_acc[47] += nl; st_acc[49] += ne; st_acc[50] += __popcll(__ballot(chk0)) + __popcll(__ballot(chk1)); }
      if (action == 1) return true;
      if (ntw < 1) return false;
      if (ne == 0) {
        r.winner = (uint32_t)__builtin_amdgcn_readfirstlane((int)twv);
        return true;
      }
      // exclusions: the jp-th of the remaining ties, in the window (tie jp + k in lane k of twv)
      const int64_t jp = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(h3.y) << 32) |
                                   (uint32_t)__builtin_amdgcn_readfirstlane(h3.x));
      r.T -= ne;
      if (r.T < jp) return false;
      for (int k = 0; k < ntw; ++k) {
        const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)twv, k);
        const bool ex = __ballot(tie && w == x) != 0;
        const int c = __popcll(__ballot(tie && w < x));
        if (!ex && c == k) { r.winner = x; return true; }
      }
      return false;
    };

    while (!err) {
      SPM(2);
      if (SPLIT) {
        int cut_at;
        if (vshare) {
          const v4i32 ctl = ld_ctl();   // rb_req, vend (unused), verified, cut_at
          if (const int rq = ctl.x) {
            if (!rollback(rq - 1)) break;
            continue;
          }
          ver = ctl.z;
          cut_at = ctl.w;
          // a Reserve that needs the host's cpuset selection ends the batch right after its pod; else every pod
          // before the end of the decisions verified
          if (cut_at >= 0 && ver > cut_at) { committed = cut_at + 1; host_cut = true; break; }
          if (ver == end_at) { committed = ver; break; }
        } else {
          cut_at = ld_acq(&s_cut_at);
          const int vs = verify_step(cut_at);
          if (vs == 1) {
            if (!rollback(ver)) break;
            continue;
          }
          if (vs == 2) break;
        }
        SPM(55);   // split: verification
        if (ps_slot >= 0) {   // the last fresh slot's batch-start scores, then the snapshot the prep wave reads
          flush_fresh();
          WAVE_FENCE();
        }
        if (lane == 0 && ld_acq(&s_snap) != q) st_rel(&s_snap, q);
        SPM(27);   // verification, fresh slot's scores
        if (q >= end_at || q - ver >= lag || cut_at >= 0 || ld_acq(&s_prep_done) <= q || ld_acq(&s_reprep)) {
          if (ST) {   // diagnostics: why wave 0 waits (first reason that holds)
            const int why = q >= end_at ? 0 : q - ver >= lag ? 1 : cut_at >= 0 ? 2 : ld_acq(&s_reprep) ? 3 : 4;
            st_acc[56 + why] += 1;
          }
          if (++spins > SP_SPIN_LIMIT) { err = true; err_code = 2; break; }
          if (const int we = ld_acq(&s_werr)) { err = true; err_code = we; break; }
          if (vshare) verify_try();
          else __builtin_amdgcn_s_sleep(1);
          if (q >= end_at) SPM(23);   // waiting at the batch's end
          continue;
        }
        spins = 0;
        if (ST) st_acc[35] += nd;
        const int p = q;
        Dc r;
        if (!apply_late(p, r)) {   // the prep wave records p again over the exact state (every decision before p)
          if (ST) st_acc[48] += 1;
          if (lane == 0) st_rel(&s_reprep, p + 1);
          SPM(11);
          continue;
        }
        if (ST) st_acc[10] += r.slowpath ? 1 : 0;
        SPM(19);   // the prep record, the late landings
        if (r.action == 0 && (int32_t)r.winner < 0) { r.action = 2; r.end_why = 4; }
        if (r.action == 2) {   // stop deciding here: the batch ends at p once everything before it is verified
          end_at = p;
          end_why = r.end_why;
          continue;
        }
        record(p, r);
        ++q;
        continue;
      }
      const v4i32 ctl = ld_ctl();   // rb_req, vend, verified, cut_at
      // ------------------------------------------------ a rollback the verifier requested: to pod v
      if (const int rq = ctl.x) {
        if (!rollback(rq - 1)) break;
        continue;
      }
      {   // the verifier has verified every pod before the batch's end (or a host cut)
        const int vend = ctl.y;
        if (vend >= 0) {
          committed = vend;
          host_cut = ld_acq(&s_vcut) != 0;
          break;
        }
      }
      SPM(27);   // rollback / batch-end checks
      // ------------------------------------------------ decide pod q
      if (q >= end_at || q - ctl.z >= lag || ctl.w >= 0) {
        if (++spins > SP_SPIN_LIMIT) { err = true; err_code = 2; break; }
        if (const int we = ld_acq(&s_werr)) { err = true; err_code = we; break; }
        sp_sleep();
        if (q >= end_at) SPM(23);   // waiting at the batch's end
        continue;
      }
      spins = 0;
      if (ST) st_acc[35] += nd;
      const int p = q;
      const Hdr h = nh;
      Dc r;
      decide_core(p, h, nh, true, flush_fresh, nd, dn0, dn1, pv0, pv1, Tag<false>{}, r);
      if (r.action == 4) {   // diagnostics (no speculation): wait for the pending rows
        if (++spins > SP_SPIN_LIMIT) { err = true; err_code = 3; break; }
        sp_sleep();
        continue;
      }
      const bool full_row = r.action == 3;
      if (ST) st_acc[10] += full_row ? 1 : 0;
      if (full_row) {
        full_row_resolve(p, h.tbv, r, nd, dn0, dn1, hash_ok);
        SPM(11);
      }
      if (r.action == 0 && (int32_t)r.winner < 0) { r.action = 2; r.end_why = 4; }
      if (r.action == 2) {   // stop deciding here: the batch ends at p once everything before it is verified
        end_at = p;
        end_why = r.end_why;
        if (lane == 0) st_rel(&s_end_at, p);
        continue;
      }
      record(p, r);
      ++q;
    }
    if (!err && committed > 0) {   // every committed pod's Reserve is in place before the waves stop
      uint32_t w = 0;
      for (;;) {
        bool all = true;
        for (int qq = lane; qq < committed; qq += 64) all = all && ld_acq(&resv[qq]) != 0;
        if (!__ballot(!all)) break;
        if (++w > SP_SPIN_LIMIT) { err = true; err_code = 4; break; }
        if (const int we = ld_acq(&s_werr)) { err = true; err_code = we; break; }
        sp_sleep();
      }
      // the last pod's Reserve can cut after the verifier has passed it (nothing waits for its re-scoring)
      const int ca = ld_acq(&s_cut_at);
      if (!err && ca >= 0 && ca < committed) {
        committed = ca + 1;
        host_cut = true;
      }
    }
    if (ST) st_acc[12] = __builtin_amdgcn_s_memtime() - st_t0;
    if (lane == 0) {
      s_committed = committed;
      s_endwhy = committed < B ? (end_why << 16 | (host_cut ? 0x8000 : 0) | (end_at & 0xfff)) : 0;
      s_hostcut = host_cut ? 1 : 0;
      s_nd = nd;
      if (err) s_err = err_code ? err_code : 9;
      st_rel(&s_finish, 1);
    }
  } else if (SPLIT && wv == SP_W_PREP) {
    // ===================================================== prep =====================================================
    // Pod p's selectHost over the snapshot of the decisions published in s_snap (slot table in LDS), up to
    // SP_PREPQ - 1 pods ahead of wave 0, into the PrepRec ring; wave 0 applies the landings after the snapshot.
    __builtin_amdgcn_s_setprio(3);
    int pn = 0;   // the next pod in queue order (its header prefetched in nh)
    Hdr nh;
    load_hdr(0, nh);
    int hash_nd = -1;   // the node -> slot hash holds the snapshot's first hash_nd slots (full-row resolution)
    uint32_t spins = 0;
    for (;;) {
      if (ld_acq(&s_stop)) {   // a rollback: park; resume at its pod
        if (lane == 0) __atomic_fetch_add(&s_parked, 1, __ATOMIC_ACQ_REL);
        while (ld_acq(&s_stop) && !ld_acq(&s_finish)) sp_sleep();
        pn = ld_acq(&s_rb_at);
        if (pn < B) load_hdr(pn, nh);
        hash_nd = -1;
        SPM(2);
        continue;
      }
      if (ld_acq(&s_finish)) break;
      const int rq = ld_acq(&s_reprep);
      int p = pn;
      bool wait = false;
      if (rq) {   // wave 0 asks for pod rq - 1 over the exact state: once the snapshot holds every decision before it
        p = rq - 1;
        wait = ld_acq(&s_snap) != p;
      } else {
        wait = pn >= B || pn >= ld_acq(&s_decided) + prep_ahead;
      }
      if (wait) {
        if (++spins > SP_SPIN_LIMIT) {
          if (lane == 0) __atomic_store_n(&s_werr, 10, __ATOMIC_RELEASE);
          break;
        }
        if (vprep) verify_try();   // its idle time: the decided pods' verification
        else if (pn >= B && !rq) sp_sleep();
        else __builtin_amdgcn_s_sleep(1);
        SPM(2);
        continue;
      }
      spins = 0;
      const int qs = ld_acq(&s_snap);
      int nds = 0;
      if (qs > 0) nds = dec[qs - 1].nd_before + ((dec[qs - 1].flags & SP_FRESH) ? 1 : 0);
      const uint32_t dn0 = lane < nds ? (uint32_t)L.slot_node[lane] : 0xffffffffu;
      const uint32_t dn1 = lane + 64 < nds ? (uint32_t)L.slot_node[lane + 64] : 0xffffffffu;
      const int32_t pv0 = lane < nds ? L.slot_pv[lane] : -1;
      const int32_t pv1 = lane + 64 < nds ? L.slot_pv[lane + 64] : -1;
      Hdr h = nh;
      if (rq) load_hdr(p, h);
      Dc r;
      decide_core(p, h, nh, !rq, [] {}, nds, dn0, dn1, pv0, pv1, Tag<true>{}, r);
      const bool exact = qs == p;
      if (r.action == 3 && exact) {
        bool ok = hash_nd == nds;
        full_row_resolve(p, h.tbv, r, nds, dn0, dn1, ok);
        hash_nd = nds;
      }
      int act = r.action;
      if (act == 0 && (int32_t)r.winner < 0) { act = 2; r.end_why = 4; }
      if (act >= 3 || (!exact && (act == 2 || r.slowpath))) act = 5;
      if (act == 0 && r.ntw == 0) {   // (forced / full-row decisions) the window is the winner alone
        r.ntw = 1;
        r.twv = lane == 0 ? r.winner : 0xffffffffu;
      }
      PrepRec& o = L.prq[p % SP_PREPQ];
      if (lane == 0) {
        o.pod = p;
        o.q_s = qs;
        o.nd_s = nds;
        o.action = act;
        o.M = r.M;
        o.Mclean = r.Mclean;
        o.F = r.F;
        o.ntw = r.ntw;
        o.end_why = r.end_why;
        o.slow = r.slowpath ? 1 : 0;
        o.T_lo = (int32_t)r.T;
        o.T_hi = (int32_t)(r.T >> 32);
        o.jp_lo = (int32_t)r.jp;
        o.jp_hi = (int32_t)(r.jp >> 32);
      }
      if (lane < SP_KW) o.tw[lane] = r.twv;
      if (lane < nds) o.sf[lane] = (uint8_t)r.sf0;
      if (lane + 64 < nds) o.sf[lane + 64] = (uint8_t)r.sf1;
      WAVE_FENCE();
      if (rq) {
        if (lane == 0) st_rel(&s_reprep, 0);
      } else {
        if (lane == 0) st_rel(&s_prep_done, p + 1);
        ++pn;
      }
      if (ST) st_acc[9] += 1;
      SPM(0);
    }
  } else if (!SPLIT && wv == SP_W_VERIFY) {
    // ==================================================== verify ====================================================
    // pod v stands iff every row pending at its decision now scores below its maximum for it (and every row whose
    // batch-start score was unknown scored below it at batch start); the rows it excluded that are feasible join its
    // Feasible count. A miss asks wave 0 to roll back to v. Verifying v needs the re-scoring of every pod before it
    // (rescored[]), which also means their Reserves (and batch-start jobs) are complete.
    sp_prio((a.dbg >> 8) & 3u);
    int v = 0, wm = 0;
    uint32_t spins = 0;
    for (;;) {
      if (ld_acq(&s_stop)) {   // a rollback: park; wave 0 resets the verified count to the rollback's pod
        if (lane == 0) __atomic_fetch_add(&s_parked, 1, __ATOMIC_ACQ_REL);
        while (ld_acq(&s_stop) && !ld_acq(&s_finish)) sp_sleep();
        v = ld_acq(&s_verified);
        wm = v;
        SPM(2);
        continue;
      }
      if (ld_acq(&s_finish)) break;
      if (ld_acq(&s_rb_req) || ld_acq(&s_vend) >= 0) { sp_sleep(); SPM(2); continue; }   // wave 0 acts on it
      const int qd = ld_acq(&s_decided);
      while (wm < qd && ld_acq(&rescored[wm])) ++wm;
      bool moved = false, req = false;
      while (v < qd && v <= wm) {
        // nothing past a host cut is verified: the batch ends after the cut pod whatever the later decisions
        const int cut_v = ld_acq(&s_cut_at);
        if (cut_v >= 0 && v > cut_v) break;
        const DecRec d = dec[v];
        int mis = 0, fadd = 0;
        if ((d.pend0 >> lane) & 1ull) {
          const int sc = dsc[v * SB + lane];
          mis |= sc >= 0 && sc >= d.M;
          fadd += sc >= 0;
        }
        if ((d.pend1 >> lane) & 1ull) {
          const int sc = dsc[v * SB + 64 + lane];
          mis |= sc >= 0 && sc >= d.M;
          fadd += sc >= 0;
        }
        // unknown batch-start scores (several shards): known now (the creating pod is complete); the decision counted
        // the node as clean and unlisted
        if ((d.unk0 >> lane) & 1ull) {
          const int so = dso[v * SB + lane];
          mis |= so >= 0 && so >= d.M;
          fadd -= so >= 0;
        }
        if ((d.unk1 >> lane) & 1ull) {
          const int so = dso[v * SB + 64 + lane];
          mis |= so >= 0 && so >= d.M;
          fadd -= so >= 0;
        }
        if (__ballot(mis)) {
          if (lane == 0) st_rel(&s_rb_req, v + 1);
          req = true;
          break;
        }
        const int F = d.F + wave_sum(fadd);
        if (lane == 0) final_F[v] = F;
        ++v;
        moved = true;
        if (lane == 0) st_rel(&s_verified, v);
      }
      if (req) { SPM(1); continue; }
      if (moved) SPM(1);
      {   // a Reserve that needs the host's cpuset selection ends the batch right after its pod
        const int cut_at = ld_acq(&s_cut_at);
        if (cut_at >= 0 && v > cut_at) {
          if (lane == 0) { s_vcut = 1; st_rel(&s_vend, cut_at + 1); }
          continue;
        }
      }
      if (v == ld_acq(&s_end_at)) {   // every pod before the end of the decisions is verified
        if (lane == 0) st_rel(&s_vend, v);
        continue;
      }
      if (moved) { spins = 0; continue; }
      if (++spins > SP_SPIN_LIMIT) {
        if (lane == 0) __atomic_store_n(&s_werr, 8, __ATOMIC_RELEASE);
        break;
      }
      sp_sleep();
      SPM(2);
    }
  } else if (sp_reserve_index(wv) >= 0) {
    // =================================================== Reserve ===================================================
    const int wr = sp_reserve_index(wv);   // this wave's pods: q % SP_NRES == wr
    sp_prio((a.dbg >> 4) & 3u);
    uint64_t* s_cpuset_w = s_cpuset[wr];
    int32_t& s_aff_w = s_aff[wr];
    Job* jq = jobq + wr * SP_JOBQ;
    int32_t& jq_tail = s_jq_tail[wr];
    int32_t& jq_head = s_jq_head[wr];
    int f_kind = 0, f_region = 0, f_off = 0, f_size = 8;
    const void* f_src = nullptr;
    if (lane < ROW_I64) { f_kind = 1; f_src = m.c64(kRowCol[lane]); f_off = lane * 8; }
    else if (lane == ROW_I64) { f_kind = 2; f_src = m.c32(C_FREE_PODS); f_off = offsetof(Row, free_pods); f_size = 4; }
    else if (lane == ROW_I64 + 1) { f_kind = 2; f_src = m.c32(C_DFLAGS); f_off = offsetof(Row, dflags); f_size = 4; }
    else if (lane == ROW_I64 + 2) { f_kind = 4; f_off = offsetof(Row, node); }
    else if (numa_on) {
      // CpuStateDev's 11 words (C_CPU_UN0 .. C_CPU_XC1), meta, topo; lanes 32..61 the NUMA row
      if (lane >= 20 && lane < 31) { f_kind = 1; f_src = m.c64(C_CPU_UN0 + (lane - 20)); f_region = 1; f_off = (lane - 20) * 8; }
      else if (lane == 31) { f_kind = 2; f_src = m.c32(C_CPU_META); f_region = 1; f_off = offsetof(CpuStateDev, meta); f_size = 4; }
      else if (lane == 62) { f_kind = 2; f_src = m.c32(C_TOPO_DEV); f_region = 1; f_off = offsetof(CpuStateDev, topo); f_size = 4; }
      else if (lane == 63) { f_kind = 3; f_src = a.aff; f_region = 2; f_size = 4; }
      else if (lane >= 32 && lane < 32 + NUMA_I64) {
        f_kind = 1; f_src = m.c64(C_ZCAP_CPU0 + (lane - 32)); f_off = offsetof(Row, nr) + (lane - 32) * 8;
      } else if (lane >= 50 && lane < 50 + NUMA_I32) {
        f_kind = 2; f_src = m.c32(C_NFLAGS + (lane - 50)); f_off = offsetof(Row, nr.nflags) + (lane - 50) * 4; f_size = 4;
      }
    }
    // one load per lane of the fetch map for a fresh winner row of pod qq
    auto fetch = [&](int qq, uint32_t node) -> int64_t {
      int64_t vv = 0;
      if (f_kind == 1) vv = reinterpret_cast<const int64_t*>(f_src)[node];
      else if (f_kind == 2) vv = reinterpret_cast<const int32_t*>(f_src)[node];
      else if (f_kind == 3) {   // the Filter-time affinity, known for the own shard's unpatched rows (-1: recomputed)
        const uint8_t b = node - a.own0 < a.own1 - a.own0
                              ? reinterpret_cast<const uint8_t*>(f_src)[(size_t)qq * a.ld + (node - a.own0)]
                              : AFF_RECOMPUTE;
        vv = b == AFF_RECOMPUTE ? (int64_t)-1 : (int64_t)b;
      }
      else if (f_kind == 4) vv = (int64_t)node;
      return vv;
    };
    int q = wr, pf_q = -1;   // pf_q: the pod whose fresh winner row is in flight in pf_v
    int64_t pf_v = 0;
    uint32_t spins = 0;
    // room for n more jobs in this wave's ring (it is the only producer); false: a rollback or the end intervened
    auto room = [&](int n) -> bool {
      uint32_t w = 0;
      while (jq_tail - ld_acq(&jq_head) + n > SP_JOBQ) {
        if (ld_acq(&s_stop) || ld_acq(&s_finish)) return false;
        if (++w > SP_SPIN_LIMIT) {
          if (lane == 0) __atomic_store_n(&s_werr, 7, __ATOMIC_RELEASE);
          return false;
        }
        sp_sleep();
      }
      return true;
    };
    for (;;) {
      if (ld_acq(&s_stop)) {   // rollback: park until wave 0 has repaired the state, resume at its pod of our parity
        if (lane == 0) __atomic_fetch_add(&s_parked, 1, __ATOMIC_ACQ_REL);
        while (ld_acq(&s_stop) && !ld_acq(&s_finish)) sp_sleep();
        const int v = ld_acq(&s_rb_at);
        q = v + ((wr - v) & (SP_NRES - 1));
        pf_q = -1;
        continue;
      }
      if (ld_acq(&s_finish)) break;
      const int cut_now = ld_acq(&s_cut_at);
      if (q >= ld_acq(&s_decided) || (cut_now >= 0 && q > cut_now)) {
        if (++spins > SP_SPIN_LIMIT) {
          if (lane == 0) __atomic_store_n(&s_werr, 5, __ATOMIC_RELEASE);
          break;
        }
        sp_sleep();
        if (q == 0) SPM(26);   // waiting for the batch's first decision
        SPM(6);
        continue;
      }
      spins = 0;
      SPM(6);
      const DecRec d = dec[q];
      const PodVec& pk = pods(q);
      if (d.flags & SP_FITERR) {
        if (lane == 0) {
          a.out[q] = PlacementDev{-1, (uint32_t)d.F, 0, 0, 0, 0, 0, {0, 0, 0, 0}, {0, 0, 0, 0}};
          __atomic_store_n(&rescored[q], 1, __ATOMIC_RELEASE);
          __atomic_store_n(&resv[q], 1, __ATOMIC_RELEASE);
        }
        WAVE_FENCE();
        if (vshare && !vprep) verify_try();
        q += SP_NRES;
        continue;
      }
      const int slot = d.slot;
      const uint32_t winner = (uint32_t)d.winner;
      const bool fresh = d.flags & SP_FRESH;
      if (fresh) {   // the row: one load per lane (issued one pod ahead when pod q was already decided), then LDS
        const int64_t vv = pf_q == q ? pf_v : fetch(q, winner);
        pf_q = -1;
        const int qn = q + SP_NRES;   // this wave's next pod
        if (qn < ld_acq(&s_decided)) {   // prefetch its fresh winner row
          const DecRec& dn = dec[qn];
          if ((dn.flags & (SP_FRESH | SP_FITERR)) == SP_FRESH) { pf_v = fetch(qn, (uint32_t)dn.winner); pf_q = qn; }
        }
        if (f_kind) {
          unsigned char* dst = f_region == 0 ? reinterpret_cast<unsigned char*>(&drows[slot])
                             : f_region == 1 ? reinterpret_cast<unsigned char*>(&cst[slot])
                                             : reinterpret_cast<unsigned char*>(&s_aff_w);
          if (f_size == 8) *reinterpret_cast<int64_t*>(dst + f_off) = vv;
          else *reinterpret_cast<int32_t*>(dst + f_off) = (int32_t)vv;
        }
        if (lane == 0) has_row[slot] = 1;
        SPM(21);   // fresh row fetch
      } else {
        // the slot's previous version must be fully re-scored before its row changes
        bool stop = false;
        while (ld_acq(&done_ver[slot]) < d.prev_pend) {
          if (ld_acq(&s_stop) || ld_acq(&s_finish)) { stop = true; break; }
          sp_sleep();
        }
        if (stop) continue;
        SPM(22);   // landed-again slot: wait for its previous re-scoring
      }
      const int nlater = B - (q + 1);
      const int njobs = (nlater + 63) / 64;
      const bool xjob = (d.flags & SP_OFFSHARD) && njobs > 0;
      // ring room for this pod's jobs before the Reserve changes anything (a rollback may end the wait; it only grows)
      if (!room(njobs + (xjob ? 1 : 0))) continue;
      if (xjob) {   // another shard's row: its batch-start job goes first, ahead of the row's re-scoring jobs
        if (lane == 0) {
          jobs_left[q] = njobs;
          jobs_all[q] = njobs + 1;
          const int t = jq_tail;
          jq[t % SP_JOBQ] = Job{slot, q, -1, (int32_t)winner};
          __atomic_store_n(&jq_tail, t + 1, __ATOMIC_RELEASE);
        }
        WAVE_FENCE();
      }
      if (lane == 0 && (!fresh || !numa_on)) s_aff_w = -1;
      WAVE_FENCE();
      {   // undo log: the slot's state before this Reserve
        UndoRec& u = undo[q % SP_LAG];
        const uint64_t* src = reinterpret_cast<const uint64_t*>(&drows[slot]);
        uint64_t* dst = reinterpret_cast<uint64_t*>(&u.row);
        for (int i = lane; i < (int)(sizeof(Row) / 8); i += 64) dst[i] = src[i];
        const uint64_t* s2 = reinterpret_cast<const uint64_t*>(&cst[slot]);
        uint64_t* d2 = reinterpret_cast<uint64_t*>(&u.cs);
        for (int i = lane; i < (int)(sizeof(CpuStateDev) / 8); i += 64) d2[i] = s2[i];
        if (lane == 0) u.slot = slot;
      }
      WAVE_FENCE();
      SPM(15);   // row fetch + undo log
      Row& dr_ = drows[slot];
      int cut = 0;
      {
        const Row dr = dr_;
        const uint32_t nf = dr.nr.nflags;
        const bool maybe_rb = (pk.numa & PN_BIND) || (((nf >> NF_BIND_SHIFT) & 3u) && (pk.req_keys & 1u) && pk.req[0]);
        const bool numa_reserve =
            numa_on && !(pk.numa & (PN_SKIP | PN_PREFAIL)) && (maybe_rb || ((nf >> NF_POLICY_SHIFT) & 3u));
        NumaOut no{};
        if (numa_reserve)
          no = numa_eval<true, false, true>(dr.nr, pk, a.pf, SlotsLds{dr, m}, a.pf.enabled & 0x10u, false, s_aff_w);
        SPM(16);   // topology staging + the Reserve's NUMA Allocate (numa_eval)
        if (lane == 0) {
          PlacementDev pl{(int32_t)winner, (uint32_t)d.F, (int64_t)d.M, (uint32_t)d.T, (d.flags & SP_SLOW) ? 1u : 0u,
                          0, 0, {0, 0, 0, 0}, {0, 0, 0, 0}};
          if (numa_reserve) {
            const bool rb = no.flags & GS_PLACED_CPUSET;
            if (no.reason) pl.flags |= PL_RESERVE_FAILED;
            if (rb || ((nf >> NF_POLICY_SHIFT) & 3u)) {
              pl.flags |= no.flags;
              pl.zkeys = no.zkeys;
#pragma unroll
              for (int z = 0; z < 4; ++z) { pl.zcpu[z] = no.zcpu[z]; pl.zmem[z] = no.zmem[z]; }
              if (nf & NF_TOPO_VALID) {
                uint32_t f2 = dr.nr.nflags2;
#pragma unroll
                for (int z = 0; z < 4; ++z) {
                  const bool zc = no.zkeys >> z & 1u, zm = no.zkeys >> (4 + z) & 1u;
                  if (!zc && !zm) continue;
                  dr_.nr.zraw_cpu[z] = dr.nr.zraw_cpu[z] + no.zcpu[z];
                  dr_.nr.zraw_mem[z] = dr.nr.zraw_mem[z] + no.zmem[z];
                  f2 |= (1u << (NF2_ENTRY_SHIFT + z)) | (zc ? 1u << (NF2_ACPU_SHIFT + z) : 0u) |
                        (zm ? 1u << (NF2_AMEM_SHIFT + z) : 0u);
                }
                dr_.nr.nflags2 = f2;
              }
              if (rb) {
                CpuStateDev& cs = cst[slot];
                if (cpuset_on_device(cs, pk)) {   // (the topology's TopoDev is read from HBM: scalar loads)
                  if (cpuset_reserve(a.topos + cs.topo, (GS_LDS CpuStateDev*)&cs, pk, nf, no.zkeys,
                                     no.zcpu[0], no.zcpu[1], no.zcpu[2], no.zcpu[3], (GS_LDS NumaRow*)&dr_.nr,
                                     (GS_LDS uint64_t*)s_cpuset_w)) {
                    pl.flags |= PL_DEVICE_CPUSET;
#pragma unroll
                    for (int j = 0; j < 4; ++j) pl.cpuset[j] = s_cpuset_w[j];
                  } else {
                    pl.flags |= PL_RESERVE_FAILED;
                  }
                } else {
                  cut = 1;
                }
              }
            }
          }
          a.out[q] = pl;
          for (int s = 0; s < 7; ++s) dr_.free[s] = dr.free[s] - pk.req[s];
          dr_.nzfree[0] = dr.nzfree[0] - pk.nz[0];
          dr_.nzfree[1] = dr.nzfree[1] - pk.nz[1];
          dr_.free_pods = dr.free_pods - 1;
          dr_.la_free[0] = dr.la_free[0] - pk.est[0];
          dr_.la_free[1] = dr.la_free[1] - pk.est[1];
          if (pk.flags & PF_PROD) {
            dr_.la_pfree[0] = dr.la_pfree[0] - pk.est[0];
            dr_.la_pfree[1] = dr.la_pfree[1] - pk.est[1];
          }
        }
      }
      cut = __builtin_amdgcn_readlane(cut, 0);
      WAVE_FENCE();
      SPM(17);   // lane 0: placement record, zone split, cpuset_reserve, assume deltas
      if (pf_q != q + SP_NRES && q + SP_NRES < ld_acq(&s_decided)) {   // our next pod was decided meanwhile: its row
        const DecRec& dn = dec[q + SP_NRES];
        if ((dn.flags & (SP_FRESH | SP_FITERR)) == SP_FRESH) {
          pf_v = fetch(q + SP_NRES, (uint32_t)dn.winner);
          pf_q = q + SP_NRES;
        }
      }
      // a pod whose cpuset the host must select ends the batch after it: published before its re-scoring can complete
      // (the verifier passes a pod only once the pod before it is re-scored); the first such pod in queue order wins
      if (lane == 0 && cut) {
        int cur = ld_acq(&s_cut_at);
        while ((cur < 0 || q < cur) &&
               !__atomic_compare_exchange_n(&s_cut_at, &cur, q, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
        }
      }
      WAVE_FENCE();
      // ---- the row's re-scoring: hint table of its new state, jobs of 64 later pods
      if (njobs == 0) {
        if (lane == 0) {
          __atomic_store_n(&done_ver[slot], q, __ATOMIC_RELEASE);
          __atomic_store_n(&rescored[q], 1, __ATOMIC_RELEASE);
        }
      } else {
        if (lane == 0) {
          if (!xjob) {
            jobs_left[q] = njobs;
            jobs_all[q] = njobs;
          }
          int t = jq_tail;
          for (int j = 0; j < njobs; ++j, ++t) jq[t % SP_JOBQ] = Job{slot, q, j, 0};
          __atomic_store_n(&jq_tail, t, __ATOMIC_RELEASE);
        }
      }
      WAVE_FENCE();
      if (lane == 0) __atomic_store_n(&resv[q], 1, __ATOMIC_RELEASE);
      WAVE_FENCE();
      if (vshare && !vprep && njobs == 0) verify_try();
      q += SP_NRES;
      SPM(5);
    }
  } else {
    // ============================================== re-scoring jobs ==============================================
    uint32_t spins = 0;
    const int ri = SPLIT ? wv - SP_RS0 : sp_rescore_index(wv);   // split: waves 4-7
    sp_prio((a.dbg >> 6) & 3u);
    int ring = ri % SP_NRES;
    for (;;) {
      if (ld_acq(&s_stop)) {
        if (lane == 0) __atomic_fetch_add(&s_parked, 1, __ATOMIC_ACQ_REL);
        while (ld_acq(&s_stop) && !ld_acq(&s_finish)) sp_sleep();
        continue;
      }
      if (ld_acq(&s_finish)) break;
      // a job from either Reserve wave's ring (the preferred one alternating). The entry is read before the head moves
      // past it: until then its producer cannot reuse the slot
      int h = -1;
      Job jl{0, 0, 0, 0};
      if (lane == 0) {
        for (int i = 0; i < SP_NRES && h < 0; ++i) {
          const int k = (ring + i) % SP_NRES;
          const int hd = __atomic_load_n(&s_jq_head[k], __ATOMIC_ACQUIRE);
          if (hd < __atomic_load_n(&s_jq_tail[k], __ATOMIC_ACQUIRE)) {
            jl = jobq[k * SP_JOBQ + hd % SP_JOBQ];
            int expect = hd;
            if (__atomic_compare_exchange_n(&s_jq_head[k], &expect, hd + 1, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE))
              h = k;
          }
        }
      }
      h = __builtin_amdgcn_readfirstlane(h);
      ring = (ring + 1) % SP_NRES;
      if (h < 0) {
        if (++spins > SP_SPIN_LIMIT) {
          if (lane == 0) __atomic_store_n(&s_werr, 6, __ATOMIC_RELEASE);
          break;
        }
        sp_sleep();
        SPM(8);
        continue;
      }
      spins = 0;
      SPM(8);
      const Job jb{__builtin_amdgcn_readfirstlane(jl.slot), __builtin_amdgcn_readfirstlane(jl.q),
                   __builtin_amdgcn_readfirstlane(jl.range), __builtin_amdgcn_readfirstlane(jl.tbl)};
      HintTable& tab = tables[ri];
      if (jb.range < 0) {
        // batch-start job (several shards): another shard's fresh row as it stood at batch start — the HBM mirror,
        // written back only at the kernel's end — evaluated for every later pod: its dso entries
        const uint32_t node = (uint32_t)__builtin_amdgcn_readfirstlane(jb.tbl);
        Row rr;
        load_row(m, node, true, numa_on, rr);
        for (int s = 3; s < 7; ++s) rr.free[s] = m.c64(C_FREE_CPU + s)[node];
        if (numa_on && ((rr.nr.nflags >> NF_POLICY_SHIFT) & 3u)) hint_table_fill(tab, rr.nr, zone_avail(rr.nr), lane);
        WAVE_FENCE();
        for (int q2 = jb.q + 1 + lane; q2 < B; q2 += 64) dso[q2 * SB + jb.slot] = (int16_t)row_score(rr, pods(q2), a.pf, m, &tab);
        WAVE_FENCE();
        if (lane == 0 && __atomic_fetch_sub(&jobs_all[jb.q], 1, __ATOMIC_ACQ_REL) == 1)
          __atomic_store_n(&rescored[jb.q], 1, __ATOMIC_RELEASE);
        WAVE_FENCE();
        SPM(7);
        continue;
      }
      const Row rr = drows[jb.slot];
      if (numa_on && ((rr.nr.nflags >> NF_POLICY_SHIFT) & 3u)) hint_table_fill(tab, rr.nr, zone_avail(rr.nr), lane);
      WAVE_FENCE();
      SPM(9);   // re-scoring job: row copy + hint table
      const int q2 = jb.q + 1 + jb.range * 64 + lane;
      if (ST) {
        // diagnostics: could the job's lanes have been skipped? Per later pod q2, from the row's batch-start score so
        // (an upper bound of every later version's under LeastAllocated on a row without a NUMA policy): 0 infeasible
        // at batch start, 1 feasible below q2's lowest listed level (its lists hold >= q2 + 1 nodes), 2 needed exactly,
        // 3 lists too short for the bound. Regions 30.. (no policy) and 40.. (policy rows) of the re-scoring waves.
        const bool pol = numa_on && ((rr.nr.nflags >> NF_POLICY_SHIFT) & 3u);
        int cat = -1;
        if (q2 < B) {
          const int so = dso[q2 * SB + jb.slot];
          const LevelHdr* h = hdr_ptr(a, 0, q2);
          const LevelExt* x = reinterpret_cast<const LevelExt*>(a.xbase + (size_t)a.bmax * LCAP * 4 +
                                                                (size_t)a.bmax * sizeof(LevelHdr)) + q2;
          const int nl = min(x->nlev, LEVALL);
          int tot = 0, lo = -1;
          for (int j = 0; j < nl; ++j) {
            tot += j < MAXLEV ? h->count[j] : x->count[j - MAXLEV];
            lo = j < MAXLEV ? h->score[j] : x->score[j - MAXLEV];
          }
          cat = so < 0 ? 0 : tot < q2 + 1 ? 3 : so < lo ? 1 : 2;
        }
        const uint64_t act = __ballot(q2 < B), c0 = __ballot(cat == 0), c1 = __ballot(cat == 1), c2 = __ballot(cat == 2),
                       c3 = __ballot(cat == 3);
        const int base = pol ? 40 : 30;
        st_acc[base] += 1;
        st_acc[base + 1] += __popcll(act);
        st_acc[base + 2] += __popcll(c0);
        st_acc[base + 3] += __popcll(c1);
        st_acc[base + 4] += __popcll(c2);
        st_acc[base + 5] += __popcll(c3);
        st_acc[base + 6] += (c1 | c2 | c3) == 0 ? 1 : 0;   // every lane infeasible at batch start
        st_acc[base + 7] += (c2 | c3) == 0 ? 1 : 0;        // no lane needs the exact score
      }
      if (q2 < B) dsc[q2 * SB + jb.slot] = (int16_t)row_score(rr, pods(q2), a.pf, m, &tab);
      WAVE_FENCE();
      int fin = 0;
      if (lane == 0) {
        if (__atomic_fetch_sub(&jobs_left[jb.q], 1, __ATOMIC_ACQ_REL) == 1)
          __atomic_store_n(&done_ver[jb.slot], jb.q, __ATOMIC_RELEASE);
        if (__atomic_fetch_sub(&jobs_all[jb.q], 1, __ATOMIC_ACQ_REL) == 1) {
          __atomic_store_n(&rescored[jb.q], 1, __ATOMIC_RELEASE);
          fin = 1;
        }
      }
      WAVE_FENCE();
      if (vshare && !vprep && __builtin_amdgcn_readfirstlane(fin)) verify_try();
      if (ST) st_acc[10] += 1;
      SPM(7);
    }
  }
  __syncthreads();
  // ---- a host cut ends the batch after its pod, but the other Reserve wave may have reserved a later decided pod
  // meanwhile: those Reserves are undone (newest first) before the write-back
  if (wv == 0 && s_hostcut && !s_err) {
    for (int qq = s_decided - 1; qq >= s_committed; --qq) {
      if (!resv[qq] || (dec[qq].flags & SP_FITERR)) continue;
      const UndoRec& u = undo[qq % SP_LAG];
      const int sl = u.slot;
      const uint64_t* src = reinterpret_cast<const uint64_t*>(&u.row);
      uint64_t* dst = reinterpret_cast<uint64_t*>(&drows[sl]);
      for (int i = lane; i < (int)(sizeof(Row) / 8); i += 64) dst[i] = src[i];
      const uint64_t* s2 = reinterpret_cast<const uint64_t*>(&u.cs);
      uint64_t* d2 = reinterpret_cast<uint64_t*>(&cst[sl]);
      for (int i = lane; i < (int)(sizeof(CpuStateDev) / 8); i += 64) d2[i] = s2[i];
      WAVE_FENCE();
    }
  }
  __syncthreads();
  // ---- write back the fetched dirty rows; final Feasible counts. After an expired wait nothing is written back and
  // nothing is committed: the HBM mirror keeps its batch-start state, which is the host's (it applies no placement)
  const int nd = s_err ? 0 : s_nd, committed = s_err ? 0 : s_committed;
  for (int e = tid; e < nd * ROW_I64; e += SP_THREADS) {
    const int s = e / ROW_I64, j = e % ROW_I64;
    if (has_row[s] && row_word_mutable(j)) m.c64(kRowCol[j])[drows[s].node] = reinterpret_cast<const int64_t*>(&drows[s])[j];
  }
  for (int s = tid; s < nd; s += SP_THREADS)
    if (has_row[s]) m.c32(C_FREE_PODS)[drows[s].node] = drows[s].free_pods;
  constexpr int NW = 8 + 11 + 11 + 1;
  if (numa_on)
    for (int e = tid; e < nd * NW; e += SP_THREADS) {
      const int sl = e / NW, j = e % NW;
      if (!has_row[sl]) continue;
      const uint32_t node = drows[sl].node;
      if (j < 8) m.c64(C_ZRAW_CPU0 + j)[node] = (&drows[sl].nr.zraw_cpu[0])[j];
      else if (j < 19) m.c32(C_NFLAGS2 + (j - 8))[node] = reinterpret_cast<const int32_t*>(&drows[sl].nr.nflags2)[j - 8];
      else if (j < 30) m.c64(C_CPU_UN0 + (j - 19))[node] = reinterpret_cast<const int64_t*>(&cst[sl])[j - 19];
      else m.c32(C_CPU_META)[node] = (int32_t)cst[sl].meta;
    }
  for (int i = tid; i < committed; i += SP_THREADS) a.out[i].feasible = (uint32_t)final_F[i];
  if (ST && lane == 0)   // per wave: region wv of SP_STRIDE entries
    for (int i = 0; i < SP_NST; ++i)
      if (st_acc[i])
        atomicAdd(reinterpret_cast<unsigned long long*>(&a.stamps[wv * SP_STRIDE + i]), (unsigned long long)st_acc[i]);
  if (tid == 0) {
    a.committed[0] = committed;
    a.committed[1] = (committed == B && !s_hostcut && !s_err) ? 1 : 0;
    a.committed[2] = s_endwhy;   // diagnostics: why a batch ended early (GS_DEBUG_CUTS)
    a.committed[3] = s_err;
    a.committed[4] = (int32_t)(__builtin_amdgcn_s_memrealtime() - rt0);
  }
}

// With an exclusive commit CU the workgroup declares the CU's whole LDS, and the kernels that run beside it (the
// next batch's eval pass) declare a few bytes (eval_lds_bytes), so none of their waves is placed on the commit's CU.
template <bool STAMPS, bool SPLIT>
static size_t spec_launch_bytes(int npods) {
  if (!commit_cu_exclusive()) return spec_smem_bytes(npods);
  static const size_t dyn = [] {
    hipFuncAttributes fa{};
    size_t st = 0;
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(commit_spec_kernel<STAMPS, SPLIT>)) == hipSuccess)
      st = fa.sharedSizeBytes;   // the variant's static LDS
    return std::max(spec_smem_bytes(MAX_BATCH), (size_t)LDS_PER_CU - st);
  }();
  return dyn;
}

template <bool STAMPS, bool SPLIT>
static void spec_launch(const CommitArgs& a, hipStream_t st) {
  const size_t bytes = spec_launch_bytes<STAMPS, SPLIT>(a.npods);
  hipLaunchKernelGGL((commit_spec_kernel<STAMPS, SPLIT>), dim3(1), dim3(SP_THREADS), bytes, st, a);
}

hipError_t launch_commit_spec(const CommitArgs& a, hipStream_t st) {
  // the split pipeline (GS_SPEC_SPLIT, dbg bit 16): one shard, speculation on
  // and batches of GS_SPEC_SPLIT_MINB pods or more (default 32): a short batch has no selection to hide behind the
  // prep wave, only its start-up
  static const int min_b = getenv("GS_SPEC_SPLIT_MINB") ? atoi(getenv("GS_SPEC_SPLIT_MINB")) : 32;
  const bool split = ((a.dbg >> 16) & 1u) && a.nranks <= 1 && !(a.dbg & 1u) && a.npods >= min_b;
  if (a.stamps) {
    if (split) spec_launch<true, true>(a, st);
    else spec_launch<true, false>(a, st);
  } else {
    if (split) spec_launch<false, true>(a, st);
    else spec_launch<false, false>(a, st);
  }
  return hipGetLastError();
}

template <bool STAMPS, bool SPLIT>
static hipError_t spec_attr() {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(commit_spec_kernel<STAMPS, SPLIT>),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)spec_launch_bytes<STAMPS, SPLIT>(MAX_BATCH));
}

hipError_t set_commit_spec_attributes() {
  hipError_t e = spec_attr<false, false>();
  if (e == hipSuccess) e = spec_attr<false, true>();
  if (e == hipSuccess) e = spec_attr<true, false>();
  if (e == hipSuccess) e = spec_attr<true, true>();
  return e;
}

#undef SPM

}  // namespace gs

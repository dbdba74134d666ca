// gs_kernels.h — launch interface of the HIP kernels (host <-> device contract).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gs_cpuset_dev.h"
#include "gs_layout.h"

namespace gs {

constexpr int MAX_BATCH = 128;       // pods per device pass (commit-kernel LDS budget)
constexpr int MAX_RANKS = 8;
constexpr int MAXLEV = 8;            // score levels listed per (pod, shard)
constexpr int LCAP = 2048;           // listed nodes per (pod, shard)
constexpr int XCAP = 256;            // listed nodes per (pod, shard) when the lists are all-gathered for the speculative
                                     // commit (the exchange block is 8x smaller; merged: <= MAX_RANKS x XCAP = LCAP)
constexpr int PODS_PER_BLOCK = 16;   // eval kernel: pods per workgroup (grid.y = ceil(B / 16))
constexpr int MAX_SCORE_LIMIT = 2047; // cand kernel keeps one histogram per wave in LDS
constexpr int ROW_WORDS = NUM_I64_COLS + NUM_I32_COLS;  // staging row: i64 columns, then i32 widened
constexpr uint8_t AFF_RECOMPUTE = 0xFF;   // aff[][] entry the Reserve recomputes (a row patched after the eval pass)

// The HBM mirror: column c of the int64 table starts at i64 + c*npad.
struct MirrorView {
  int64_t* i64;
  int32_t* i32;
  uint32_t npad;
#ifdef __HIPCC__
  __host__ __device__
#endif
  int64_t* c64(int c) const { return i64 + (size_t)c * npad; }
#ifdef __HIPCC__
  __host__ __device__
#endif
  int32_t* c32(int c) const { return i32 + (size_t)c * npad; }
};

// Per (pod, shard) candidate summary: the top score levels of the shard's row, each with its full
// node list (node index order). Every feasible node of the shard with a score above `next` is listed.
struct LevelHdr {
  int32_t nlev;              // listed levels
  int32_t feasible;          // feasible nodes of the shard for this pod
  int32_t next;              // highest score of a feasible node that is NOT listed (-1: none)
  int32_t total;             // listed nodes
  int32_t score[MAXLEV];     // descending
  int32_t count[MAXLEV];     // nodes per level; level j starts at sum(count[0..j))
};
static_assert(sizeof(LevelHdr) == 80, "LevelHdr layout");

// Levels 8.. of the same summary (up to LEVALL levels in all; the lists hold their nodes after level 7's): read by
// the speculative commit kernel, whose pods then find k+1 listed nodes without the full-row path (C3: the top 8
// levels hold a median of 14 nodes, the top 24 at least 136).
constexpr int LEVALL = 32, LEVX = LEVALL - MAXLEV;
struct LevelExt {
  int32_t nlev;              // listed levels in all (<= LEVALL)
  int32_t next;              // highest score of a feasible node that is NOT listed (-1: none)
  int32_t score[LEVX];       // levels MAXLEV.. (descending; -1 past nlev)
  int32_t count[LEVX];
};
static_assert(sizeof(LevelExt) == 200, "LevelExt layout");

struct PlacementDev {   // gs_placement + the NodeNUMAResource Reserve the device applied / the host must apply
  int32_t node;
  uint32_t feasible;
  int64_t score;
  uint32_t ties;
  uint32_t flags;        // GS_PLACED_* | PL_* below
  uint32_t zkeys;        // NUMA allocation by hint: bit z = zone z cpu allocated, bit 4+z = memory
  uint32_t pad;
  int64_t zcpu[4], zmem[4];
  uint64_t cpuset[4];    // with PL_DEVICE_CPUSET: the CPUs the commit kernel allocated
};
enum : uint32_t {
  PL_DEVICE_CPUSET = 0x40000000u,   // cpuset chosen and applied on the device (else: host takeCPUs, batch cut)
  PL_RESERVE_FAILED = 0x80000000u,  // Reserve failed after a feasible Filter: the host fails loudly
  PL_INTERNAL_FLAGS = PL_DEVICE_CPUSET | PL_RESERVE_FAILED,
};

struct CommitArgs {
  MirrorView m;
  const PodVec* pods;
  const uint64_t* seq;
  int npods;
  int nranks;
  uint32_t shard_size;       // ceil(N / nranks): shard of node i = i / shard_size
  const uint8_t* xbase;      // rank r block at xbase + r*xblock: [npods_max x LCAP u32 lists | LevelHdr x npods_max |
                             //  LevelExt x npods_max]
  size_t xblock;
  int bmax;                  // pods per block layout (lists/hdrs are laid out for bmax pods)
  Profile pf;
  uint64_t seed;
  int32_t forced_node;       // >= 0: pod 0 was resolved by the exact full-row path
  int32_t forced_score;
  int64_t forced_ties;
  int32_t forced_feasible;
  PlacementDev* out;
  int32_t* committed;
  uint64_t* stamps;          // diagnostics: per-phase s_memtime cycle sums (nullptr: normal build)
  const TopoDev* topos;      // registered topologies, bit-plane form (cpuset Reserve on the device)
  const uint8_t* aff;        // [pod][ld] Filter-time affinity of NUMA-policy nodes of the own shard (eval_numa_kernel)
  uint32_t ld;
  uint32_t own0, own1;       // this rank's shard [own0, own1)
  const int16_t* S;          // batch-start score rows (one shard only: in-kernel full-row resolution; else nullptr)
  const int16_t* S_own;      // this rank's batch-start score rows (batch-start scores of fresh own-shard rows)
  const int32_t* prev;       // speculative pass: the previous batch's committed[4]; run only if prev[1] == 1
  // node sampling (gs_config.sample_nodes, one shard): window_k = numFeasibleNodesToFind(N) (0 = every node);
  // the batch starts at nextStartNodeIndex `start` (prev[2] for a speculative pass) and leaves it in committed[2]
  uint32_t window_k;
  uint32_t start;
  uint32_t nnodes;
  uint32_t dbg;              // diagnostics: bit 0 = the speculative commit waits for every pending row (no speculation)
  int32_t* tb;               // [npods x TB_N] selectHost tie-break records of each pod (speculative commit scratch)
  const int32_t* xerr;       // several shards: nonzero = the all-gathered blocks' exchange tags disagree (merge_levels)
};
// tiebreak_position(seed, seq, T) as a lookup: entries 0..TB_N-2 are the positions the reservoir walk visits
// (ascending, independent of T; INT32_MAX past the walk's end), entry TB_N-1 the largest T the entries decide
constexpr int TB_N = 32;

hipError_t set_kernel_attributes();
hipError_t launch_node_prep(const MirrorView& m, uint32_t n0, uint32_t n1, int64_t now, int32_t filter_expired,
                            int32_t has_exp, int64_t exp_ns, hipStream_t st);
// the same for the rows idx[0..n) (after a delta update rewrote them)
hipError_t launch_node_prep_idx(const MirrorView& m, const uint32_t* idx, uint32_t n, int64_t now, int32_t filter_expired,
                                int32_t has_exp, int64_t exp_ns, hipStream_t st);
// NodeNUMAResource profiles: numa_idx lists the shard's nodes with a NUMA topology policy (ascending)
hipError_t launch_eval(const MirrorView& m, const PodVec* pods, int npods, const Profile& pf, uint32_t n0, uint32_t n1,
                       int16_t* S, uint32_t ld, int prod_cols, const uint32_t* numa_idx, uint32_t numa_n,
                       uint8_t* aff, hipStream_t st, hipStream_t st2 = nullptr, hipEvent_t fork = nullptr,
                       hipEvent_t join = nullptr,
                       const MirrorView* slab = nullptr);
// the previous batch's winner rows of this shard re-evaluated for every pod of this batch (its eval pass ran beside
// the previous batch's commit)
hipError_t launch_patch(const MirrorView& m, const PodVec* pods, int npods, const Profile& pf, uint32_t n0, uint32_t n1,
                        int16_t* S, uint32_t ld, int prod_cols, uint8_t* aff, const PlacementDev* prev_out,
                        const int32_t* prev_committed, int prev_npods, hipStream_t st);
hipError_t launch_eval_full(const MirrorView& m, const PodVec* pods, int npods, const Profile& pf, uint32_t N,
                            int16_t* scores, uint16_t* codes, int16_t* plugin, int prod_cols, hipStream_t st);
void set_cand_stamps(uint64_t* p);   // diagnostics: cand_kernel phase cycles (nullptr: off)
// lcap: listed nodes per pod (<= LCAP), also the lists' stride
// The previous batch's landed rows, re-evaluated by cand_kernel's block k for pod k before its histogram (a pass
// behind a batch whose commit wrote those rows back: the eval pass ran on their state before it); on = 0: none.
struct CandPatch {
  MirrorView m;
  const PodVec* pods;
  Profile pf;
  uint32_t n0, n1;
  int prod_cols, on;
  uint8_t* aff;
  const PlacementDev* prev_out;
  const int32_t* prev_committed;
  // stale levels (on = 0, cand overlapped with the previous batch's commit): extra = listed nodes beyond pod k's k+1
  // (the previous batch's landed rows may leave the levels), hist = [pod][max_score + 1] the row's score histogram out
  int extra;
  uint32_t* hist;
};
// split_scratch (cand_split_scratch_bytes()): a short batch (<= CS_MAXB pods, no patch) spreads each row over up to
// CS_GMAX slices (cs_hist / cs_pick / cs_list kernels, GS_CAND_SPLIT=0 disables); nullptr: cand_kernel always
constexpr int CS_GMAX = 64, CS_MAXB = 32;
size_t cand_split_scratch_bytes();
hipError_t launch_cand(int16_t* S, uint32_t ld, uint32_t len, uint32_t n0, int npods, int max_score, int lcap,
                       uint32_t* lists, LevelHdr* hdrs, LevelExt* ext, hipStream_t st, const CandPatch* patch = nullptr,
                       uint32_t* split_scratch = nullptr);
// The previous batch's landed rows folded into stale levels (cand_kernel with cp.extra / cp.hist, before that batch's
// commit ended): the rows re-evaluated (S, aff patched as by cand_kernel's patch), the histogram updated, the levels
// re-picked and each listed level rewritten as its stale nodes minus the landed rows plus the landed rows now at it
hipError_t launch_fix_levels(int16_t* S, uint32_t ld, int npods, int max_score, int lcap, uint32_t* lists,
                             LevelHdr* hdrs, LevelExt* ext, const CandPatch& cp, hipStream_t st);
// Every all-gathered block ends with the sender's exchange tag: which exchange of the context's sequence it is (a
// count every rank advances identically), at which call site, for which batch. A rank whose sequence diverged from
// the others' (a different number of collectives, or another call site) is detected by every rank on the first
// exchange that pairs mismatched calls, which then fails on all of them (GS_ECOMM) instead of hanging one rank in a
// collective the others never enter.
struct XTag {
  uint32_t magic;
  uint32_t site;             // XSITE_*
  uint64_t seq;              // exchanges on the context so far (this one included)
  uint64_t batch;            // batch passes launched on the context so far
  int32_t rank;
  uint32_t bytes;            // the block's size (tag included)
};
static_assert(sizeof(XTag) == 32, "XTag layout");
constexpr uint32_t XTAG_MAGIC = 0x31585347u;   // "GSX1"
enum : uint32_t { XSITE_LEVELS = 1, XSITE_ROWSTAT = 2, XSITE_SELECT = 3, XSITE_SCORES = 4, XSITE_RUNS = 5 };
constexpr int32_t COMMIT_ERR_XTAG = 90;   // committed[3]: the level exchange's tags disagree (nothing committed)
constexpr int XERR_TAGS = 8;   // merge_levels_kernel's xerr: [0] verdict, [1] first mismatch kept, [8..] its R tags
constexpr size_t XERR_BYTES = 4 * XERR_TAGS + sizeof(XTag) * MAX_RANKS;
// tag -> dst (RCCL: written on the stream right before the all-gather, so the tag travels with the block)
hipError_t launch_write_tag(uint8_t* dst, const XTag& t, hipStream_t st);
// several shards: per pod, the all-gathered rank blocks' levels merged into one block of the single-rank layout (the
// speculative commit's input). Block 0 also compares the R blocks' tags (at xblock - sizeof(XTag)): xerr[0] = 0 when
// they name the same exchange, else 1 + the first rank that differs from rank 0 (the commit then commits nothing).
hipError_t launch_merge_levels(const uint8_t* xin, size_t xblock, int nranks, int npods, int bmax, int lstride,
                               uint8_t* xout, int32_t* xerr, hipStream_t st);
// several shards, score-row exchange (the default; GS_XCHG=levels: the level lists above): rank r's all-gathered block
// is [b x pld int16 scores | b x pld affinity bytes | ... | XTag] over its nodes [r*per, min(N, (r+1)*per)); the R blocks
// are written into the full-width score rows S[k][node] (stride ld) and affinities of the batch. Block 0 checks the R
// blocks' tags into xerr like merge_levels_kernel (the commit then commits nothing on a mismatch).
hipError_t launch_unpack_scores(const uint8_t* xin, size_t xblock, int nranks, int npods, uint32_t per, uint32_t pld,
                                uint32_t N, int16_t* S, uint8_t* aff, uint32_t ld, int32_t* xerr, hipStream_t st);
size_t commit_smem_bytes(int B);
bool commit_spec_selected(uint32_t window_k);   // the speculative commit kernel runs (else pipelined / lockstep)
hipError_t launch_commit(const CommitArgs& a, hipStream_t st);        // window_k > 0: lockstep kernel
// GS_COMMIT_EXCL=1: the commit's workgroup holds a CU of its own: it declares the whole LDS of the CU and the eval
// pass that overlaps it declares eval_lds_bytes(), so the dispatcher never places eval waves beside it. Measured
// neutral on C3 (commit 0.705 vs 0.708 ms per batch): off by default.
constexpr uint32_t LDS_PER_CU = 160u * 1024u;
bool commit_cu_exclusive();
size_t eval_lds_bytes();
hipError_t launch_commit_spec(const CommitArgs& a, hipStream_t st);   // speculative pipeline (gs_commit_spec.hip)
hipError_t set_commit_spec_attributes();
hipError_t launch_row_stats(const int16_t* S, uint32_t len, RowStat* out, hipStream_t st);
hipError_t launch_row_select(const int16_t* S, uint32_t len, int score, int64_t target, uint32_t n0, int32_t* out,
                             hipStream_t st);
struct ScatterPrep {   // node_prep_kernel's arguments, fused into the scatter
  int64_t now;
  int32_t filter_expired, has_exp;
  int64_t exp_ns;
};
hipError_t launch_scatter_rows(const MirrorView& m, const uint32_t* idx, const int64_t* rows, uint32_t nrows,
                               hipStream_t st, const ScatterPrep* prep = nullptr);
int64_t host_tiebreak_position(uint64_t seed, uint64_t seq, int64_t T);
// diagnostics (gs_probe.hip): cycles of one pair evaluation as the commit kernel runs it
hipError_t launch_probe(int mode, const MirrorView& m, const Profile& pf, const PodVec* pods, int npods,
                        const uint32_t* nodes, const int32_t* pod_of, uint32_t n, int prod_cols, int32_t* scores,
                        uint64_t* cycles, hipStream_t st);
hipError_t launch_merge_probe(const gs_merge_case* cases, int n, gs_merge_result* out, hipStream_t st);

}  // namespace gs

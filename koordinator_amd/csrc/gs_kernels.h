// gs_kernels.h — launch interface of the HIP kernels (host <-> device contract).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "gs_layout.h"

namespace gs {

constexpr int CAND_CAP = 256;                                   // candidate-list capacity per (pod, shard)
constexpr int MAX_BATCH = 128;                                  // pods per device pass (commit LDS budget)
constexpr int MAX_RANKS = 8;
constexpr int ROW_WORDS = NUM_I64_COLS + NUM_I32_COLS;          // staging row: i64 columns, then i32 columns widened

struct MirrorView {
  int64_t* i64[NUM_I64_COLS];
  int32_t* i32[NUM_I32_COLS];
};

struct PlacementDev {   // layout == gs_placement minus flags
  int32_t node;
  uint32_t feasible;
  int64_t score;
  uint32_t ties;
  uint32_t flags;
};

struct CommitArgs {
  MirrorView m;
  const PodVec* pods;
  const uint64_t* seq;
  int npods;
  int nranks;
  const uint64_t* lists;     // [rank][pod][CAND_CAP]
  const CandHdr* hdrs;       // [rank][pod]
  size_t list_stride;        // pods per rank block in `lists`
  size_t hdr_stride;
  Profile pf;
  uint64_t seed;
  int32_t forced_node;       // >= 0: pod 0 was resolved by the exact full-row path
  int32_t forced_score;
  int64_t forced_ties;
  int32_t forced_feasible;
  PlacementDev* out;
  int32_t* committed;
};

hipError_t set_kernel_attributes();
hipError_t launch_node_prep(const MirrorView& m, uint32_t n0, uint32_t n1, int64_t now, int32_t filter_expired,
                            int32_t has_exp, int64_t exp_ns, hipStream_t st);
hipError_t launch_eval(const MirrorView& m, const PodVec* pods, int npods, const Profile& pf, uint32_t n0, uint32_t n1,
                       int16_t* S, uint32_t ld, int prod_cols, hipStream_t st);
hipError_t launch_eval_full(const MirrorView& m, const PodVec* pods, int npods, const Profile& pf, uint32_t N,
                            int16_t* scores, uint16_t* codes, int16_t* plugin, int prod_cols, hipStream_t st);
hipError_t launch_cand(const int16_t* S, uint32_t ld, uint32_t len, uint32_t n0, int npods, int max_score,
                       uint64_t* lists, CandHdr* hdrs, hipStream_t st);
size_t cand_smem_bytes(int max_score);
size_t commit_smem_bytes(int B, int nranks);
hipError_t launch_commit(const CommitArgs& a, hipStream_t st);
hipError_t launch_row_stats(const int16_t* S, uint32_t len, RowStat* out, hipStream_t st);
hipError_t launch_row_select(const int16_t* S, uint32_t len, int score, int64_t target, uint32_t n0, int32_t* out,
                             hipStream_t st);
hipError_t launch_scatter_rows(const MirrorView& m, const uint32_t* idx, const int64_t* rows, uint32_t nrows,
                               hipStream_t st);
int64_t host_tiebreak_position(uint64_t seed, uint64_t seq, int64_t T);

}  // namespace gs

// gs_commit.hip — the sequential commit of a batch on the device (gfx950): the batch's pods in queue order,
// each one selectHost over its score levels and the rows earlier pods of the batch landed on, then assume +
// Reserve ([upstream] scheduleOne: selectHost, assume; LoadAware / NodeNUMAResource Reserve).
//
// For pod p the effective score of a node is its batch-start score (S, summarized per shard by the listed
// levels of cand_kernel) unless an earlier pod of the batch landed on it ("dirty"): dirty rows live in LDS and
// their scores for every later pod are re-evaluated exactly (dso = batch-start score, dsc = current score). The
// max M is valid when it exceeds every shard's highest unlisted score (`next`); otherwise one shard resolves
// the pod from its whole score row and several shards cut the batch there. Ties at M are ordered by node
// index across shards (shards are contiguous ranges).
//
// One persistent workgroup of 4 waves with fixed roles, pipelined by one pod (period p = pod p):
//   wave 0 (selector)  selectHost of pod p, fetch of the winner row, Reserve, the hint table of the row's new
//                      state, and that row's current score for pod p+1 — the one re-score pod p+1's selection
//                      needs before the next period;
//   waves 1-3          the current scores of the row pod p-1 landed on, for pods p+1.. (their selections come
//                      one period later or more), and the prefetch of pod p+1's level headers, list heads and
//                      tie-break positions into LDS.
// A workgroup barrier closes every period. Wave 0 waits inside a period only when pod p lands on the row pod p-1
// landed on: waves 1-3 are re-scoring that row and must finish before the Reserve changes it.
// Node sampling (window_k > 0) keeps the lockstep commit_kernel of gs_kernels.hip.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_eval_dev.h"

namespace gs {

constexpr int PIPE_PL = 32;    // prefetched list-head entries per (pod, shard)
constexpr int PIPE_RSN = 32;   // prefetched tie-break positions per pod
constexpr int RS_WAVES = 3;    // re-scoring waves
constexpr int RS_CAP = 1 << 30;

// tie-break positions R = {1, floor(j/U_0)+1, ...} of a pod (tiebreak_position's stream) up to RS_CAP; n < 0:
// truncated after -n entries (a T beyond the last entry takes the loop)
__device__ __forceinline__ void rset_fill(int32_t* out, int32_t* n_out, uint64_t seed, uint64_t seq) {
  const uint64_t key = mix64(seed ^ mix64(seq));
  int64_t j = 1;
  int n = 0;
  out[n++] = 1;
  bool complete = false;
  for (uint64_t i = 0; n < PIPE_RSN; ++i) {
    const uint64_t h = mix64(key + i);
    const double u = (double)((h >> 11) + 1) * 0x1.0p-53;
    const double x = (double)j / u;
    if (!(x < 4.0e18)) { complete = true; break; }
    const int64_t jn = (int64_t)floor(x) + 1;
    if (jn > RS_CAP) { complete = true; break; }
    j = jn;
    out[n++] = (int32_t)j;
  }
  *n_out = complete ? n : -n;
}

template <bool ST>
__global__ void __launch_bounds__(256) commit_pipe_kernel(CommitArgs a) {
  extern __shared__ __align__(16) unsigned char cm[];
  const int B = a.npods;
  const int R = a.nranks;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  const MirrorView& m = a.m;
  const bool numa_on = (a.pf.enabled & 0x30u) != 0;
  // ---- LDS: pod vectors (136-B stride: re-scoring lanes read different pods), dirty rows, scores, hash, CPU state
  auto pods = [&](int i) -> PodVec& { return *reinterpret_cast<PodVec*>(cm + (size_t)i * POD_STRIDE); };
  Row* drows = reinterpret_cast<Row*>(cm + (size_t)B * POD_STRIDE);
  int16_t* dsc = reinterpret_cast<int16_t*>(drows + B);   // [pod][slot] current score
  int16_t* dso = dsc + B * B;                               // [pod][slot] batch-start score
  const size_t hoff = ((size_t)B * POD_STRIDE + (size_t)B * sizeof(Row) + (size_t)B * B * 4 + 15) & ~(size_t)15;
  int32_t* hkey = reinterpret_cast<int32_t*>(cm + hoff);   // node -> slot (open addressing)
  int32_t* hval = hkey + HASH;
  CpuStateDev* cst = reinterpret_cast<CpuStateDev*>(hval + HASH);
  // prefetched per pod (parity of the pod): level headers, list heads, tie-break positions
  __shared__ LevelHdr hsh[2][MAX_RANKS];
  __shared__ uint32_t plh[2][MAX_RANKS][PIPE_PL];
  __shared__ int32_t rset[2][PIPE_RSN], rset_n[2];
  __shared__ uint64_t sseq[MAX_BATCH];
  // wave 0 selection scratch
  __shared__ int32_t sh_score[MAX_RANKS * MAXLEV], sh_dec[MAX_RANKS * MAXLEV];   // several shards: decrements
  __shared__ Row orow[2];                 // batch-start copy of a fresh row outside this rank's shard (by parity)
  __shared__ TopoDev s_topo;              // topology of the last cpuset Reserve (bit-plane form)
  __shared__ HintTable s_ht[2], s_hto[2];  // new state / batch-start state of the winner row (by parity)
  __shared__ uint64_t s_cpuset[4];
  __shared__ int32_t s_aff;               // Filter-time affinity of the pair (fresh own-shard row; -1 unknown)
  // hand-off between the roles (by parity of the pod): the slot pod p landed on (-1 none), its batch-start
  // scores are evaluated (fresh row outside the shard), stop after this period, re-scoring rounds done
  __shared__ int32_t s_wslot[2], s_weval[2];
  __shared__ int32_t s_stop, s_rdone;
  __shared__ int32_t s_committed, s_hostcut, s_nd;

  // speculative pass queued behind another batch: only if that one committed every pod with nothing left for
  // the host (committed[1] == 1); otherwise a no-op (committed = -1) the host discards
  if (a.prev && a.prev[1] != 1) {
    if (tid == 0) { a.committed[0] = -1; a.committed[1] = 0; a.committed[3] = 0; }
    return;
  }

  // ---- prologue: pods, hash, pod 0's prefetch
  uint64_t st_acc[27] = {};
  uint64_t st_last = ST ? __builtin_amdgcn_s_memtime() : 0;
// (diagnostic build: nothing moves across a stamp, and a phase's outstanding memory operations complete inside it)
#define STAMP(i)                                    \
  do {                                              \
    if (ST) {                                       \
      __builtin_amdgcn_sched_barrier(0);            \
      __builtin_amdgcn_s_waitcnt(0);                \
      uint64_t t_ = __builtin_amdgcn_s_memtime();   \
      st_acc[i] += t_ - st_last;                    \
      st_last = t_;                                 \
      __builtin_amdgcn_sched_barrier(0);            \
    }                                               \
  } while (0)
  for (int i = tid; i < B; i += 256) { pods(i) = a.pods[i]; sseq[i] = a.seq[i]; }
  for (int i = tid; i < HASH; i += 256) { hkey[i] = -1; hval[i] = -1; }
  // prefetch of pod q's headers, list heads and tie-break positions into parity slot q & 1 (one wave)
  auto prefetch = [&](int q) {
    const int par = q & 1;
    for (int e = lane; e < R * 20; e += 64) {
      const int r = e / 20, w = e % 20;
      reinterpret_cast<int32_t*>(&hsh[par][r])[w] = reinterpret_cast<const int32_t*>(hdr_ptr(a, r, q))[w];
    }
    for (int e = lane; e < R * PIPE_PL; e += 64) {
      const int r = e / PIPE_PL, i = e % PIPE_PL;
      plh[par][r][i] = list_ptr(a, r, q)[i];
    }
    if (lane == 0) rset_fill(rset[par], &rset_n[par], a.seed, a.seq[q]);
  };
  if (wv == RS_WAVES) prefetch(0);
  if (tid == 0) {
    s_stop = 0;
    s_rdone = 0;
    s_wslot[0] = s_wslot[1] = -1;
    s_committed = B;
    s_hostcut = 0;
  }
  __syncthreads();

  if (wv == 0) {
    // ===================================== wave 0: the selector =====================================
    // Dirty slot s's node id lives in a register of lane s % 64 (dn0: slots 0..63, dn1: slots 64..127), so the
    // selection reads LDS in one round (level headers, the pod's scores on the dirty slots, tie-break positions,
    // the list window) and does the rest with ballots, DPP reductions and readlane broadcasts.
    uint32_t dn0 = 0xffffffffu, dn1 = 0xffffffffu;
    int nd = 0;                  // dirty slots
    int topo_id = -1;            // s_topo holds this registered topology
    const int nhl = R * MAXLEV;  // header lanes: lane = r*MAXLEV + j
    // fresh-row fetch map of this lane (loop invariant): kind 0 none, 1 i64 column, 2 i32 column, 3 the Filter-time
    // affinity byte, 4 the node index; destination region 0 the slot's row, 1 the slot's CPU state, 2 s_aff
    int f_kind = 0, f_region = 0, f_off = 0, f_size = 8;
    const void* f_src = nullptr;
    if (lane < ROW_I64) { f_kind = 1; f_src = m.c64(kRowCol[lane]); f_off = lane * 8; }
    else if (lane == ROW_I64) { f_kind = 2; f_src = m.c32(C_FREE_PODS); f_off = offsetof(Row, free_pods); f_size = 4; }
    else if (lane == ROW_I64 + 1) { f_kind = 2; f_src = m.c32(C_DFLAGS); f_off = offsetof(Row, dflags); f_size = 4; }
    else if (lane == ROW_I64 + 2) { f_kind = 4; f_off = offsetof(Row, node); }
    else if (numa_on) {
      if (lane >= 20 && lane < 26) { f_kind = 1; f_src = m.c64(C_CPU_UN0 + (lane - 20)); f_region = 1; f_off = (lane - 20) * 8; }
      else if (lane == 26) { f_kind = 2; f_src = m.c32(C_CPU_META); f_region = 1; f_off = offsetof(CpuStateDev, meta); f_size = 4; }
      else if (lane == 27) { f_kind = 2; f_src = m.c32(C_TOPO_DEV); f_region = 1; f_off = offsetof(CpuStateDev, topo); f_size = 4; }
      else if (lane == 28) { f_kind = 3; f_src = a.aff; f_region = 2; f_size = 4; }
      else if (lane >= 32 && lane < 32 + NUMA_I64) {
        f_kind = 1; f_src = m.c64(C_ZCAP_CPU0 + (lane - 32)); f_off = offsetof(Row, nr) + (lane - 32) * 8;
      } else if (lane >= 50 && lane < 50 + NUMA_I32) {
        f_kind = 2; f_src = m.c32(C_NFLAGS + (lane - 50)); f_off = offsetof(Row, nr.nflags) + (lane - 50) * 4; f_size = 4;
      }
    }
    // node ids of the dirty slots selected by two lane bitmaps, in lane order
    auto each_node = [&](uint64_t m0, uint64_t m1, auto&& fn) {
      for (uint64_t b = m0; b; b &= b - 1) fn((uint32_t)__builtin_amdgcn_readlane((int)dn0, __builtin_ctzll(b)));
      for (uint64_t b = m1; b; b &= b - 1) fn((uint32_t)__builtin_amdgcn_readlane((int)dn1, __builtin_ctzll(b)));
    };
    int committed = B;
    bool host_cut = false;
    for (int p = 0; p < B; ++p) {
      const int par = p & 1;
      STAMP(11);
      // ------------------------------------------------------------ selectHost of pod p
      // action 0 commit, 1 FitError (nothing assumed), 2 cut the batch before p
      int action = 0;
      uint32_t winner = 0xffffffffu;
      int M = -1, F = 0;
      int64_t T = 0;
      bool slowpath = p == 0 && a.forced_node >= 0;   // pod 0 resolved by the host's full-row path
      // ---- one round of LDS loads
      const int r_l = lane / MAXLEV, j_l = lane % MAXLEV;
      const int nlev_l = lane < nhl ? hsh[par][r_l].nlev : 0;
      const bool lvl = lane < nhl && j_l < nlev_l;
      const int hs = lvl ? hsh[par][r_l].score[j_l] : -1, hc = lvl ? hsh[par][r_l].count[j_l] : 0;
      const int feas_l = lane < R ? hsh[par][lane].feasible : 0, next_l = lane < R ? hsh[par][lane].next : -1;
      int sc0 = -1, so0 = -1, sc1 = -1, so1 = -1;
      if (lane < nd) { sc0 = dsc[p * B + lane]; so0 = dso[p * B + lane]; }
      if (lane + 64 < nd) { sc1 = dsc[p * B + 64 + lane]; so1 = dso[p * B + 64 + lane]; }
      const int rn = rset_n[par], rna = rn < 0 ? -rn : rn;
      const int32_t rv = lane < rna ? rset[par][lane] : 0x7fffffff;
      const int sh0 = (int)(dn0 / a.shard_size), sh1 = (int)(dn1 / a.shard_size);   // shard of each dirty node
      STAMP(12);
      // ---- listed-level decrements: a dirty row whose batch-start score is a listed level of its shard left it
      int clean = 0;
      if (R == 1) {
        int dec_l = 0;   // decrement of level `lane`
#pragma unroll
        for (int j = 0; j < MAXLEV; ++j) {
          const int sj = __builtin_amdgcn_readlane(hs, j);
          const int dj = __popcll(__ballot(so0 >= 0 && so0 == sj)) + __popcll(__ballot(so1 >= 0 && so1 == sj));
          if (lane == j) dec_l = dj;
        }
        clean = lvl ? hc - dec_l : 0;
      } else {
        if (lane < nhl) { sh_score[lane] = hs; sh_dec[lane] = 0; }
        WAVE_FENCE();
        for (int e = 0; e < 2; ++e) {
          const int so = e ? so1 : so0;
          if (so < 0) continue;
          const int base = (e ? sh1 : sh0) * MAXLEV;
          for (int j = 0; j < MAXLEV; ++j)
            if (sh_score[base + j] == so) { atomicAdd(&sh_dec[base + j], 1); break; }
        }
        WAVE_FENCE();
        clean = lvl ? hc - sh_dec[lane] : 0;
      }
      const int Md = wave_max(max(sc0, sc1));
      const int Fd = wave_sum((sc0 >= 0) - (so0 >= 0) + (sc1 >= 0) - (so1 >= 0));
      M = max(wave_max(clean > 0 ? hs : -1), Md);
      F = Fd + wave_sum(lane < R ? feas_l : 0);
      STAMP(13);
      bool full_row = false;
      if (slowpath) {
        M = a.forced_score;
        F = a.forced_feasible;
        T = a.forced_ties;
        winner = (uint32_t)a.forced_node;
      } else if (__ballot(lane < R && M <= next_l)) {
        // a shard may hold unlisted nodes at M: one shard resolves pod p from its whole row right here; with several
        // shards the batch is cut and the host resolves it (row_stats / row_select / exchange)
        if (R == 1 && a.S) full_row = true;
        else action = 2;
      } else if (M < 0) {
        action = 1;   // FitError: no feasible node anywhere
      } else {
        // ---- tie set at M: clean listed nodes + dirty rows now at M ("new") - dirty rows listed at M ("old")
        const bool nw0 = sc0 == M, nw1 = sc1 == M;
        const int ndn = __popcll(__ballot(nw0)) + __popcll(__ballot(nw1));
        const int cm_lane = (lvl && hs == M) ? clean : 0;
        T = (int64_t)wave_sum(cm_lane) + ndn;
        int64_t jp;   // tie-break position: the largest prefetched R entry <= T
        {
          const uint64_t le = __ballot(lane < rna && (int64_t)rv <= T);
          const int top = 63 - __clzll((long long)le);
          jp = __builtin_amdgcn_readlane(rv, top);
          if (rn < 0 && top == rna - 1) jp = tiebreak_position(a.seed, sseq[p], T);   // past the prefetched entries
        }
        // owning shard r*: per shard, clean listed ties + dirty rows now at M, by prefix in shard order
        int rstar = 0;
        if (R > 1) {
          int64_t before = 0;
          for (int r = 0; r < R; ++r) {
            const int here = wave_sum(r_l == r ? cm_lane : 0) + __popcll(__ballot(nw0 && sh0 == r)) +
                             __popcll(__ballot(nw1 && sh1 == r));
            if (before + here >= jp || r == R - 1) { rstar = r; break; }
            before += here;
          }
          jp -= before;
        }
        // level-M segment of r*'s list: offset = listed nodes of r* above M, len = listed nodes at M
        int off = 0, len = 0;
        for (int j = 0; j < MAXLEV; ++j) {
          const int sj = __builtin_amdgcn_readlane(hs, rstar * MAXLEV + j);
          const int cj = __builtin_amdgcn_readlane(hc, rstar * MAXLEV + j);
          if (sj < 0) break;
          if (sj == M) { len = cj; break; }
          off += cj;
        }
        const uint32_t sb = (uint32_t)rstar * a.shard_size, se = sb + a.shard_size;
        const bool in0 = dn0 >= sb && dn0 < se, in1 = dn1 >= sb && dn1 < se;
        const uint64_t new0 = __ballot(nw0 && in0), new1 = __ballot(nw1 && in1);
        const uint64_t old0 = __ballot(so0 == M && in0), old1 = __ballot(so1 == M && in1);
        const int nnew = __popcll(new0) + __popcll(new1), nold = __popcll(old0) + __popcll(old1);
        const int lo = (int)max<int64_t>(0, jp - 2 - nnew);
        const int hi = (int)min<int64_t>(len - 1, jp - 1 + nold);
        const int W = hi - lo + 1;   // <= nold + nnew + 2
        STAMP(14);
        // ---- the jp-th node of (listed level-M nodes of r* - old) U new, node order, over window L[lo..hi]
        // (list entries below PIPE_PL come from the prefetched head); window position i in lane i % 64 of chunk i / 64
        const uint32_t* L = list_ptr(a, rstar, p);
        constexpr int WCH = (2 * MAX_BATCH + 2 + 63) / 64;
        uint32_t xw[WCH];
        bool ow[WCH];
        uint32_t cand = 0xffffffffu;
        int base_old = 0;
        if (len > 0) {
#pragma unroll
          for (int c = 0; c < WCH; ++c) {
            const int i = c * 64 + lane, e = off + lo + i;
            xw[c] = 0xffffffffu;
            if (c * 64 < W && i < W) xw[c] = e < PIPE_PL ? plh[par][rstar][e] : L[e];
          }
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
        // a new node is the jp-th when its insertion point in the window decides position jp
        each_node(new0, new1, [&](uint32_t n) {
          int u = 0;   // rank among the new nodes
          each_node(new0, new1, [&](uint32_t n2) { u += n2 < n ? 1 : 0; });
          int64_t ltn = -1;   // # listed level-M nodes < n, when it can decide position jp
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
        STAMP(15);
        const uint64_t got = __ballot(cand != 0xffffffffu);
        if (!got) action = 2;   // unreachable for a valid max: cut, exact re-run on the host
        else winner = (uint32_t)__builtin_amdgcn_readlane((int)cand, __ffsll((long long)got) - 1);
        STAMP(16);
      }
      STAMP(17);
      if (ST) { st_acc[18] += full_row ? 1 : 0; st_acc[19] += action == 1 ? 1 : 0; st_acc[20] += slowpath ? 1 : 0; }
      if (full_row) {
        // ---- exact full-row resolution of pod p on the single shard: batch-start scores S[p][*] for clean nodes,
        // current scores for dirty rows; max, ties and feasible count, then the jp-th tie in node order
        // (coalesced 16-B loads, lane l holds nodes [8l, 8l+8) of each 512-node block). A dirty row's batch-start
        // score is dso (= S on the single shard), so the clean ties at a score are the raw ties minus the dirty rows
        // listed at it; the dirty-slot hash is only probed when every raw node at the row's maximum is dirty.
        const int16_t* row = a.S + (size_t)p * a.ld;
        const uint32_t len = a.own1 - a.own0;
        constexpr int VB = 8;   // blocks in flight per step
        auto load_blk = [&](uint32_t i0, int16_t (&x)[8]) {
          if (i0 + 8 <= len) {
            const uint4 v = *reinterpret_cast<const uint4*>(row + i0);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
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
        F = wave_sum(lfeas) + Fd;
        int Mc = wave_max(lmax);
        int64_t Tc = Mc >= 0 ? (int64_t)wave_sum(lmax == Mc ? lcnt : 0) - __popcll(__ballot(so0 == Mc)) -
                                   __popcll(__ballot(so1 == Mc))
                             : 0;
        if (Mc >= 0 && Tc <= 0) {   // every raw node at the maximum is dirty: the clean maximum, probing the hash
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
                if (xv >= 0 && xv >= lmax && hash_find(hkey, hval, a.own0 + b0 + 512u * u + 8u * lane + k) < 0) {
                  lcnt = xv > lmax ? 1 : lcnt + 1;
                  lmax = xv;
                }
              }
          }
          Mc = wave_max(lmax);
          Tc = Mc >= 0 ? (int64_t)wave_sum(lmax == Mc ? lcnt : 0) : 0;
        }
        M = max(Mc, Md);
        if (M < 0) {
          action = 1;
        } else {
          const uint64_t new0 = __ballot(sc0 == M), new1 = __ballot(sc1 == M);   // dirty rows now at M
          const uint64_t old0 = __ballot(so0 == M), old1 = __ballot(so1 == M);   // dirty rows listed at M in S
          T = (Mc == M ? Tc : 0) + __popcll(new0) + __popcll(new1);
          const int64_t jp = tiebreak_position(a.seed, sseq[p], T);
          // the jp-th tie in node order: raw nodes at M, less the dirty rows listed there, plus the dirty rows now at M
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
              // the block's ties: raw ties at M, less the dirty rows listed at M, plus the dirty rows now at M
              const bool in0 = dn0 - a.own0 - i0 < 512u, in1 = dn1 - a.own0 - i0 < 512u;
              const uint64_t bn0 = new0 & __ballot(in0), bn1 = new1 & __ballot(in1);
              const uint64_t bo0 = old0 & __ballot(in0), bo1 = old1 & __ballot(in1);
              const int tot = wave_sum(__popc(fl)) + __popcll(bn0) + __popcll(bn1) - __popcll(bo0) - __popcll(bo1);
              if (found == -1 && run + tot >= jp) {   // the jp-th tie is in this block: exact per-node flags
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
                const uint64_t got = __ballot(f >= 0);
                found = got ? (int64_t)__builtin_amdgcn_readlane((int)f, __ffsll((long long)got) - 1) : -2;
              }
              run += tot;
            }
          }
          if (found < 0) action = 2;
          else winner = (uint32_t)found;
          slowpath = true;
        }
        STAMP(26);
      }
      if (slowpath && action == 0 && (int32_t)winner < 0) action = 2;   // unreachable for a valid max
      STAMP(0);
      if (action == 2) {
        committed = p;
        if (lane == 0) { s_wslot[par] = -1; s_stop = 1; }
        WAVE_FENCE();
        __syncthreads();
        break;
      }
      if (action == 1) {
        if (lane == 0) {
          a.out[p] = PlacementDev{-1, (uint32_t)F, 0, 0, 0, 0, 0, {0, 0, 0, 0}, {0, 0, 0, 0}};
          s_wslot[par] = -1;
          if (p == B - 1) s_stop = 1;
        }
        WAVE_FENCE();
        STAMP(10);
        __syncthreads();
        STAMP(6);
        continue;
      }
      // ------------------------------------------------------------ fetch the winner into its dirty slot
      const uint64_t hit0 = __ballot(dn0 == winner), hit1 = __ballot(dn1 == winner);
      int slot = hit0 ? __builtin_ctzll(hit0) : hit1 ? 64 + __builtin_ctzll(hit1) : -1;
      const bool fresh = slot < 0;
      const bool own = winner >= a.own0 && winner < a.own1;
      const bool eval_so = fresh && !own;   // batch-start scores outside this rank's shard are evaluated
      if (fresh) {
        slot = nd;
        if (lane == (nd & 63)) { if (nd < 64) dn0 = winner; else dn1 = winner; }
        if (lane == 0) {   // the node -> slot hash (full-row resolution)
          uint32_t h = (winner * 2654435761u) & (HASH - 1);
          while (hkey[h] >= 0) h = (h + 1) & (HASH - 1);
          hkey[h] = (int32_t)winner;
          hval[h] = slot;
        }
        ++nd;
        // one load per lane, all issued before a single wait
        int64_t v = 0;
        if (f_kind == 1) v = reinterpret_cast<const int64_t*>(f_src)[winner];
        else if (f_kind == 2) v = reinterpret_cast<const int32_t*>(f_src)[winner];
        else if (f_kind == 3) {   // the batch-start Filter's affinity for this pair (own shard, NUMA-policy nodes)
          const uint8_t b8 = own ? reinterpret_cast<const uint8_t*>(f_src)[(size_t)p * a.ld + (winner - a.own0)]
                                 : AFF_RECOMPUTE;
          v = b8 == AFF_RECOMPUTE ? (int64_t)-1 : (int64_t)b8;   // (a patched row's: recomputed)
        } else if (f_kind == 4) v = (int64_t)winner;   // Row.node, Row.pad = 0
        // batch-start scores of the later pods on this row (own shard): S[q][winner], q = p+1 ..
        int16_t so0v = 0, so1v = 0;
        const int q0 = p + 1 + lane, q1 = q0 + 64;
        if (own && q0 < B) so0v = a.S_own[(size_t)q0 * a.ld + (winner - a.own0)];
        if (own && q1 < B) so1v = a.S_own[(size_t)q1 * a.ld + (winner - a.own0)];
        if (f_kind) {
          unsigned char* dst = f_region == 0 ? reinterpret_cast<unsigned char*>(&drows[slot])
                             : f_region == 1 ? reinterpret_cast<unsigned char*>(&cst[slot])
                                             : reinterpret_cast<unsigned char*>(&s_aff);
          if (f_size == 8) *reinterpret_cast<int64_t*>(dst + f_off) = v;
          else *reinterpret_cast<int32_t*>(dst + f_off) = (int32_t)v;
          if (eval_so && f_region == 0) {
            unsigned char* d2 = reinterpret_cast<unsigned char*>(&orow[par]);
            if (f_size == 8) *reinterpret_cast<int64_t*>(d2 + f_off) = v;
            else *reinterpret_cast<int32_t*>(d2 + f_off) = (int32_t)v;
          }
        }
        if (own && q0 < B) dso[q0 * B + slot] = so0v;
        if (own && q1 < B) dso[q1 * B + slot] = so1v;
      }
      if (lane == 0 && (!fresh || !numa_on)) s_aff = -1;   // a dirty row changed since the batch-start Filter
      WAVE_FENCE();
      STAMP(1);
      // the row pod p-1 landed on is being re-scored by waves 1-3: wait for them before changing it
      if (!fresh && p > 0 && slot == s_wslot[(p - 1) & 1]) {
        while (__atomic_load_n(&s_rdone, __ATOMIC_ACQUIRE) < RS_WAVES * (p + 1)) __builtin_amdgcn_s_sleep(1);
      }
      STAMP(2);
      Row& d = drows[slot];
      const PodVec& pk = pods(p);
      // ------------------------------------------------------------ Reserve
      if (numa_on) {   // stage the winner's topology in LDS for a device-side cpuset Reserve
        const int tp = cst[slot].topo;
        const uint32_t nfl = d.nr.nflags;
        if (tp >= 0 && tp != topo_id && !(pk.numa & (PN_SKIP | PN_PREFAIL)) &&
            ((pk.numa & PN_BIND) || ((nfl >> NF_BIND_SHIFT) & 3u))) {
          const uint64_t* src = reinterpret_cast<const uint64_t*>(a.topos + tp);
          uint64_t* dst = reinterpret_cast<uint64_t*>(&s_topo);
          for (int i = lane; i < (int)(sizeof(TopoDev) / 8); i += 64) dst[i] = src[i];
          topo_id = tp;
        }
        WAVE_FENCE();
      }
      STAMP(3);
      int cut = 0;
      {
        const Row dr = d;   // wave-uniform copy: the Reserve's pair evaluation re-reads row words
        const uint32_t nf = dr.nr.nflags;
        // Reserve returns at once unless requestCPUBind (util.go:105-122) or the node has a NUMA policy
        const bool maybe_rb = (pk.numa & PN_BIND) || (((nf >> NF_BIND_SHIFT) & 3u) && (pk.req_keys & 1u) && pk.req[0]);
        const bool numa_reserve =
            numa_on && !(pk.numa & (PN_SKIP | PN_PREFAIL)) && (maybe_rb || ((nf >> NF_POLICY_SHIFT) & 3u));
        // NodeNUMAResource Reserve (plugin.go:375-422) on the pre-assume row: the Filter-time affinity and the NUMA
        // split of Allocate (the whole wave evaluates the pair); a cpuset pod's CPUs are selected by lane 0
        // (gs_cpuset_dev.h) when the node's topology is in the device scope, else the batch ends with it and the
        // host selects them
        NumaOut no{};
        if (numa_reserve)
          no = numa_eval<true, false, true>(dr.nr, pk, a.pf, SlotsLds{dr, m}, a.pf.enabled & 0x10u, false, s_aff);
        STAMP(24);
        if (ST) st_acc[25] += (pk.numa & PN_BIND) ? 1 : 0;
        if (lane == 0) {
          PlacementDev pl{(int32_t)winner, (uint32_t)F, (int64_t)M, (uint32_t)T, slowpath ? 1u : 0u, 0, 0,
                          {0, 0, 0, 0}, {0, 0, 0, 0}};
          if (numa_reserve) {
            const bool rb = no.flags & GS_PLACED_CPUSET;
            if (no.reason) pl.flags |= PL_RESERVE_FAILED;   // cannot happen for a feasible winner
            if (rb || ((nf >> NF_POLICY_SHIFT) & 3u)) {
              pl.flags |= no.flags;
              pl.zkeys = no.zkeys;
#pragma unroll
              for (int z = 0; z < 4; ++z) { pl.zcpu[z] = no.zcpu[z]; pl.zmem[z] = no.zmem[z]; }
              if (nf & NF_TOPO_VALID) {   // resourceManager.Update -> NodeAllocation.addPodAllocation
                uint32_t f2 = dr.nr.nflags2;
#pragma unroll
                for (int z = 0; z < 4; ++z) {
                  const bool zc = no.zkeys >> z & 1u, zm = no.zkeys >> (4 + z) & 1u;
                  if (!zc && !zm) continue;
                  d.nr.zraw_cpu[z] = dr.nr.zraw_cpu[z] + no.zcpu[z];
                  d.nr.zraw_mem[z] = dr.nr.zraw_mem[z] + no.zmem[z];
                  f2 |= (1u << (NF2_ENTRY_SHIFT + z)) | (zc ? 1u << (NF2_ACPU_SHIFT + z) : 0u) |
                        (zm ? 1u << (NF2_AMEM_SHIFT + z) : 0u);
                }
                d.nr.nflags2 = f2;
              }
              if (rb) {
                CpuStateDev& cs = cst[slot];
                if (cs.topo >= 0 && cs.topo == topo_id) {
                  if (cpuset_reserve((const GS_LDS TopoDev*)&s_topo, (GS_LDS CpuStateDev*)&cs, pk, nf, no.zkeys,
                                     no.zcpu[0], no.zcpu[1], no.zcpu[2], no.zcpu[3], (GS_LDS NumaRow*)&d.nr,
                                     (GS_LDS uint64_t*)s_cpuset)) {
                    pl.flags |= PL_DEVICE_CPUSET;
#pragma unroll
                    for (int j = 0; j < 4; ++j) pl.cpuset[j] = s_cpuset[j];
                  } else {
                    pl.flags |= PL_RESERVE_FAILED;
                  }
                } else {
                  cut = 1;
                }
              }
            }
          }
          a.out[p] = pl;
          for (int s = 0; s < 7; ++s) d.free[s] = dr.free[s] - pk.req[s];
          d.nzfree[0] = dr.nzfree[0] - pk.nz[0];
          d.nzfree[1] = dr.nzfree[1] - pk.nz[1];
          d.free_pods = dr.free_pods - 1;
          d.la_free[0] = dr.la_free[0] - pk.est[0];
          d.la_free[1] = dr.la_free[1] - pk.est[1];
          if (pk.flags & PF_PROD) {
            d.la_pfree[0] = dr.la_pfree[0] - pk.est[0];
            d.la_pfree[1] = dr.la_pfree[1] - pk.est[1];
          }
        }
      }
      cut = __builtin_amdgcn_readlane(cut, 0);
      WAVE_FENCE();
      STAMP(4);
      // ------------------------------------------------------------ the new state's hint table, re-score for p+1
      const bool last = p == B - 1 || cut;
      {
        const Row rr = d;   // the row after assume + Reserve (wave-uniform)
        if (numa_on) {
          if ((rr.nr.nflags >> NF_POLICY_SHIFT) & 3u) hint_table_fill(s_ht[par], rr.nr, zone_avail(rr.nr), lane);
          if (eval_so) {
            const NumaRow no = orow[par].nr;
            if ((no.nflags >> NF_POLICY_SHIFT) & 3u) hint_table_fill(s_hto[par], no, zone_avail(no), lane);
          }
        }
        if (ST) { st_acc[22] += ((rr.nr.nflags >> NF_POLICY_SHIFT) & 3u) ? 1 : 0; st_acc[23] += fresh ? 1 : 0; }
        STAMP(21);
        if (!last) {   // the whole wave evaluates the pair (current score; batch-start score when evaluated)
          for (int it = 0; it < (eval_so ? 2 : 1); ++it) {   // one call site: one inlined copy of the evaluation
            const Row ru = it ? orow[par] : rr;
            const int32_t x = row_score_wave(ru, pods(p + 1), a.pf, m, nullptr);
            if (lane == 0) (it ? dso : dsc)[(p + 1) * B + slot] = (int16_t)x;
          }
        }
      }
      if (lane == 0) {
        s_wslot[par] = slot;
        s_weval[par] = eval_so ? 1 : 0;
        if (last) s_stop = 1;
      }
      WAVE_FENCE();
      STAMP(5);
      __syncthreads();
      STAMP(6);
      if (cut) { committed = p + 1; host_cut = true; break; }
    }
    if (lane == 0) {
      s_committed = committed;
      s_hostcut = host_cut ? 1 : 0;
      s_nd = nd;
    }
  } else {
    // ================================== waves 1-3: re-scoring and prefetch ==================================
    const int wr = wv - 1;
    for (int p = 0; p < B; ++p) {
      STAMP(7);
      if (wv == RS_WAVES && p + 1 < B) prefetch(p + 1);
      STAMP(8);
      if (p >= 1) {
        const int pr = (p - 1) & 1;
        const int s = s_wslot[pr];
        const int n = B - (p + 1);
        if (s >= 0 && n > 0) {
          const int ch = (n + RS_WAVES - 1) / RS_WAVES;
          const int q = p + 1 + wr * ch + lane;
          const int nit = s_weval[pr] ? 2 : 1;   // current scores; batch-start scores when evaluated
          for (int it = 0; it < nit; ++it) {       // one call site: one inlined copy of the evaluation
            if (lane < ch && q < B) {
              const Row rr = it ? orow[pr] : drows[s];   // wave-uniform
              (it ? dso : dsc)[q * B + s] = (int16_t)row_score(rr, pods(q), a.pf, m, it ? &s_hto[pr] : &s_ht[pr]);
            }
          }
        }
      }
      WAVE_FENCE();
      if (lane == 0) __atomic_fetch_add(&s_rdone, 1, __ATOMIC_RELEASE);
      STAMP(9);
      __syncthreads();
      STAMP(10);
      if (s_stop) break;
    }
  }
  __syncthreads();
  // ---- write back dirty rows
  const int nd = s_nd;
  for (int e = tid; e < nd * ROW_I64; e += 256) {
    const int s = e / ROW_I64, j = e % ROW_I64;
    if (row_word_mutable(j)) m.c64(kRowCol[j])[drows[s].node] = reinterpret_cast<const int64_t*>(&drows[s])[j];
  }
  for (int s = tid; s < nd; s += 256) m.c32(C_FREE_PODS)[drows[s].node] = drows[s].free_pods;
  // NUMA words Reserve changes: ZRAW (8 i64), NFLAGS2 .. ZADJ3 (11 i32), CPU state (6 i64 + meta)
  constexpr int NW = 8 + 11 + 6 + 1;
  static_assert(C_ZADJ0 + 3 - C_NFLAGS2 + 1 == 11, "NUMA i32 write-back columns contiguous");
  if (numa_on)
    for (int e = tid; e < nd * NW; e += 256) {
      const int sl = e / NW, j = e % NW;
      const uint32_t node = drows[sl].node;
      if (j < 8) m.c64(C_ZRAW_CPU0 + j)[node] = (&drows[sl].nr.zraw_cpu[0])[j];
      else if (j < 19) m.c32(C_NFLAGS2 + (j - 8))[node] = reinterpret_cast<const int32_t*>(&drows[sl].nr.nflags2)[j - 8];
      else if (j < 25) m.c64(C_CPU_UN0 + (j - 19))[node] = reinterpret_cast<const int64_t*>(&cst[sl])[j - 19];
      else m.c32(C_CPU_META)[node] = (int32_t)cst[sl].meta;
    }
  if (tid == 0) {
    a.committed[0] = s_committed;
    a.committed[1] = (s_committed == B && !s_hostcut) ? 1 : 0;
    a.committed[2] = 0;
    a.committed[3] = 0;
  }
  if (ST) {   // per-phase cycle sums of wave 0 (lane 0) and wave 1 (lane 0)
    if (tid == 0)
      for (int i = 0; i < 7; ++i) atomicAdd(reinterpret_cast<unsigned long long*>(&a.stamps[i]), st_acc[i]);
    if (tid == 0)
      for (int i = 11; i < 27; ++i) atomicAdd(reinterpret_cast<unsigned long long*>(&a.stamps[i]), st_acc[i]);
    if (tid == 64)
      for (int i = 7; i < 11; ++i) atomicAdd(reinterpret_cast<unsigned long long*>(&a.stamps[i]), st_acc[i]);
  }
#undef STAMP
}

hipError_t launch_commit_pipe(const CommitArgs& a, hipStream_t st) {
  if (a.stamps)
    hipLaunchKernelGGL(commit_pipe_kernel<true>, dim3(1), dim3(256), commit_smem_bytes(a.npods), st, a);
  else
    hipLaunchKernelGGL(commit_pipe_kernel<false>, dim3(1), dim3(256), commit_smem_bytes(a.npods), st, a);
  return hipGetLastError();
}

hipError_t set_commit_pipe_attributes() {
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(commit_pipe_kernel<false>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)commit_smem_bytes(MAX_BATCH));
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(commit_pipe_kernel<true>),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)commit_smem_bytes(MAX_BATCH));
}

}  // namespace gs

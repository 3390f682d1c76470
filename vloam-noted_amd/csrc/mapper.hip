// mapper.hip — LaserMapping::solveMapping (laser_mapping.cpp:212-814) on MI355X.
//
// One handle = B independent mapping streams; every launch below covers all of them.
// Per frame (all device resident):
//   k_stack_part/_cat  VoxelGrid of laserCloudCornerLast (0.4 m) / SurfLast (0.8 m) (:492-500),
//                      on a second stream, ahead of the frame (loam_mapper_prefetch / the
//                      solve), double-buffered by frame parity; k_stack_ds at many streams
//   k_shift_cubes      ring-buffer recentering of the 21x21x11 cube grid (:252-444), rare
//   k_frame_prep       (graph path) a queued frame's records from the frame before (initial
//                      guess :206-207, window :228-251), stack sizes, submap offsets (:448-489);
//                      no per-frame index build: every cube keeps a persistent 1 m cell
//                      index (cubeindex.h, replaces the KD-tree build :519-520), rebuilt
//                      only when its content changes (k_revox); exact 5-NN because accepted
//                      matches need all 5 neighbours within 1 m (:557, :642)
//   2 x { k_knn         exact 5-NN of every query in the cell index (:554, :633)
//         k_geom        PCA line / QR plane fit of the neighbours -> factor records (:557-699)
//         k_lm_round    all <= 5 Ceres TR-LM passes, G workgroups per stream (lm.h) }
//   k_insert_bucket    transform stacks with the final pose, assign cubes (:741-788), group
//                      the points by target cube
//   k_revox            re-VoxelGrid every changed window cube (:795-808) into the map arena,
//                      and its cell index
//   k_frame_out        (graph path) the records to the host and the frame's done word
//                      (a last-workgroup hand-off inside k_revox measured 1.5x slower: every
//                      workgroup's agent-scope release writes back L2)
//
// Map storage: per (stream, map) an append-only arena of float4 points + a cube table
// (offset, count) for the 4851 cubes; window cubes are rewritten at the arena tail every
// frame, the host compacts an arena when its tail passes half the capacity.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <array>
#include <cstring>
#include <deque>
#include <vector>

#include "common.h"
#include "device_math.h"
#include "cellhash.h"
#include "comm.h"
#include "cubeindex.h"
#include "lm.h"
#include "voxel.h"
#include "voxel_hot.h"
#include "voxel_pcl.h"

namespace loam {

constexpr int CW = 21, CH = 21, CD = 11, NCUBE = CW * CH * CD;
constexpr int WIN_MAX = 125;
constexpr int WIN_VALID_MAX = 75;
constexpr int EXTRA_CAP = 64;
// correspondence workgroups: 128 threads x 128 per stream (grid-stride) beat 256 x 64 by 3-5% at
// B = 128 and at one stream (finer scheduling of the latency-bound kNN)
constexpr int CORR_THREADS = 128;  // >= WIN_VALID_MAX (k_knn fills the window tables per thread)
constexpr int CORR_BLK = 128;
static_assert(CORR_THREADS >= WIN_VALID_MAX, "k_knn window tables");
constexpr int LM_THREADS = 256;
constexpr int LM_EBLK = 32;     // LM evaluation workgroups per stream (grid-stride)
constexpr int SUBMAP_BLOCKS = 64;
constexpr int INS_SLOTS = WIN_VALID_MAX + EXTRA_CAP;
constexpr int RQ_CLASSES = 8;  // re-VoxelGrid items by size: < 1k points, < 2k, .. < 64k, more
constexpr int MAP_ERR_SUBMAP = 4, MAP_ERR_EXTRA = 8, MAP_ERR_HASH = 16, MAP_ERR_LM_SYNC = 32,
              MAP_ERR_INDEX = 64, MAP_ERR_LIVE = 128, MAP_ERR_SORT = 256,
              MAP_ERR_STACK = 512, MAP_ERR_STACK_WAIT = 2048;

struct StreamFrame {
  double pose[7];  // in: initial guess (transformAssociateToMap); out: optimised pose
  int active;
  uint32_t epoch;  // frame counter of the handle (marks the cubes outside the window touched this frame)
  int nc_in, ns_in;
  int nc_stack, ns_stack;
  int sub_n[2];
  int optimize;
  int corner_num[2], surf_num[2];
  int valid_num;
  int window[WIN_MAX];
  int sub_off[2][WIN_MAX + 1];
  int center[3];
  int cen[3];
  int shift[3];
  int origin[3];
  uint32_t arena_tail[2];
  int arena_active[2];
  uint32_t scratch_tail[2];
  uint32_t hot_tail[2];   // exact order: the cubes' blocks of the sort scratch (pe / pa / pb / ps)
  int extra_n[2];
  int extra_list[2][EXTRA_CAP];
  int err;
  const float4* in_ptr[2];        // input clouds (mapper staging buffer or caller's HBM)
  unsigned long long cand[2];     // map points in the queries' 27-cell neighbourhoods, per round
  unsigned long long vx_bytes;    // algorithmic bytes of this frame's re-VoxelGrid + cell index
  double wodom[7];  // the frame's odometry pose q_wodom (xyzw), t_wodom
  // q_wmap_wodom, t_wmap_wodom: the frame's initial guess (:206-207) is taken with it, and k_insert_bucket
  // advances it by the frame's transformUpdate (:147-151) as the host does after the frame
  double wmap[7];
  int deferred;     // a queued frame found a recentering or compaction due: left to the host
  LmState lm[2];
};

// per-stream input of a frame in the graph path (k_frame_prep), read from page-locked host
// memory: mode 0, the host uploaded the stream records; mode 1, a frame queued behind the one
// in flight (loam_mapper_solve_async) whose records the device prepares from the frame before
struct FrameIn {
  double wodom[7];
  const float4* in_ptr[2];
  int n[2];
  int active;
  int mode;
  uint32_t epoch;
  int pad;
  unsigned long long stack_seq;  // the stack launch (launch_stacks) whose stacks the stream takes
};

// the stack VoxelGrid inputs of a stream (laser_mapping.cpp:492-500): set when its stack is
// launched (loam_mapper_prefetch or the solve), double-buffered by stack parity so that the next
// frame's stack can run beside a frame in flight
struct StackIn {
  const float4* p[2];
  int n[2];
  int active;
  int pad;
};

struct MapPose {  // by-value kernel argument: q (xyzw) + t
  double x[7];
};

struct MapperDev {
  int B;       // streams of this launch (a group of the handle's streams)
  int s0 = 0;  // first stream of the launch
  int max_in, map_cap, sub_cap, scratch_cap, max_chunks;
  float leaf[2];
  uint32_t epoch;
  StreamFrame* fr;
  float4* in_pts[2];
  float4* stack[2];
  float4* arena;  // [B][2 maps][2 arenas][map_cap]
  float4* carena; // same shape: each cube's points sorted by 1 m cell (cubeindex.h)
  uint2* ctab;    // [B][2 maps][2 arenas][4 * map_cap]: each cube's cell table
  uint2* cube_tab;  // [B][2 maps][NCUBE] (off, cnt) — current parity
  uint32_t* extra_flag;  // [B][2][NCUBE]
  int* knn_id;      // [5][B][2*max_in] neighbour ids (submap index) per query, -1: none
  size_t knn_stride;
  // factor records (SoA) [B][2*max_in]
  int* r_type;
  float* r_px;
  float* r_py;
  float* r_pz;
  double* r_a[3];
  double* r_b[3];
  float4* ins_pts;  // [B][2][max_in]
  int* ins_tag;
  float4* ins_sorted;    // [B][2][max_in] inserted points grouped by target cube (input order kept)
  uint32_t* ins_off;     // [B][2][INS_SLOTS + 1] group offsets: window slots, then extra cubes
  unsigned long long* dbg;  // [LOAM_DEBUG_COUNTERS] counters (loam_mapper_debug_counters)
  unsigned long long* pdbg;  // dbg when the phase cycle counters are on (LOAM_PHASE_COUNTERS=1), else null
  uint32_t* stable_tok;  // [B][2][NCUBE] arena offset + 1 of content known to be a VoxelGrid
                         // fixed point (re-filtering it is the identity), else 0
  float4* vx_pts;  // [B][2][scratch_cap]
  int* vx_idx;
  double* partials;  // [B][max_chunks][LM_NACC]
  uint32_t* lm_sync;   // [B][2 rounds][LM_SYNC_WORDS] (lm.h)
  double* lm_xpub;     // [B][2 rounds][8]: eval point published to the workers
  uint32_t* tickets;  // [B]
  uint32_t* lm_tick;  // [B] k_lm_eval's workgroups done (sharded: the last one reduces)
  uint32_t* rq;       // [RQ_CLASSES][rq_cap] re-VoxelGrid items ((2 s + m) INS_SLOTS + slot) by size class
  uint32_t* rq_ctl;   // [RQ_CLASSES] items per class (zeroed by the frame's first kernel)
  int rq_cap = 0;
  // sharded mode (loam_mapper_create_sharded): this rank of nrank; map points are stored by
  // the rank owning their 4 m block (comm.h, shard_owner); blk_v: voxels per block edge
  uint32_t compact_at = 0;  // an arena whose tail passed this is compacted
  uint32_t compact_due_at = 0;  // the compaction kernels' test (compact_at, or earlier: mapper_enqueue)
  // exact_voxel_order: the stack and cube VoxelGrids in PCL's summation order (voxel_pcl.h);
  // sort scratch [B][2][scratch_cap] (the stack at offset 0, the cubes from scratch_tail)
  int pcl_order = 0;
  uint64_t* pe;
  uint32_t* pa;
  uint32_t* pb;
  uint64_t* ps;
  int* pseg;  // level lists of global-memory sorts
  int rank = 0, nrank = 1, sharded = 0;
  int blk_v[2] = {1, 1};
  uint32_t* wcnt;        // [B][2][WIN_MAX] window cube counts (all-reduced over the ranks)
  struct NnRec* nn_send; // [queries of all streams] this rank's 5 nearest candidates per query
  const struct NnRec* nn_recv;  // [nrank][same]: every rank's candidates (all-gather)
  const int* q_off;      // [B] first query of stream s in nn_send
  float4* nn_xyz;        // [5][B][2*max_in] merged neighbours (k_geom input in sharded mode)
  double* pose_x;        // [nrank][B][8] every rank's optimised pose (agreement check)
  double* lm_red;        // [B][LM_NACC] this rank's normal-equation sums, then the all-reduced
  // in-process ranks (loam_comm_create_local): the persistent LM's cross-rank slots, shared by the
  // ranks (comm_peer_buffer): [2 frame parities][B][2 rounds][nrank][LM_MAX_PASSES][LM_NACC] and
  // the flags [B][2 rounds][nrank] (lm.h LmJob)
  double* lm_peer = nullptr;
  uint32_t* lm_peer_flag = nullptr;
  // ranks in separate processes (RCCL / callback comms): every rank's LM peer buffer as this
  // process maps it (ipc_peer_setup): [r] slot base, [nrank + r] flag base; each buffer holds
  // [2 frame parities][ipc_B][2 rounds][LM_MAX_PASSES][LM_NACC] f64, then flags [ipc_B][2 rounds]
  const unsigned long long* ipc_tab = nullptr;
  int ipc_B = 0;
  // few streams: the stack VoxelGrid of a (stream, map) split over stack_k workgroups by voxel
  // idx range (k_stack_part + k_stack_cat), else one workgroup (k_stack_ds)
  int stack_k = 0;
  uint2* stk_part;       // [B][2][STACK_K_MAX] (staging offset, centroids) of each range
  // the stack kernels' inputs, outputs and scratch (one stack parity: the frame's, or the next
  // frame's while this one is in flight; D.stack[m] is that parity's stack)
  const StackIn* sin;    // [B]
  int* stk_n;            // [B][2] stack sizes (copied into the frame records by k_stack_counts)
  int* stk_err;          // [B] error flags of the stack kernels (merged by k_stack_counts)
  float4* stk_pts;       // [B][2][max_in] scratch of the input-order stack filter
  int* stk_idx;          // [B][2][max_in]
  int knn_blk = CORR_BLK;  // k_knn workgroups per stream of the cell-split variant
  const FrameIn* fin = nullptr;  // [B] (page-locked host memory) the graph path's frame inputs
  unsigned long long* stk_ready = nullptr;  // the last stack launch done into this parity (k_stack_done)
  int defer_every = 0;    // tests: queued frames with epoch % defer_every == 0 are deferred
};

// one query's 5 nearest candidates on one rank (d: FLANN L2_Simple float distance, id: global
// tie-break key, xyz: the point) — the all-gathered record of the sharded kNN
struct NnRec {
  float d[5];
  int id[5];
  float x[5], y[5], z[5];
};

__device__ inline size_t sm_index(int s, int m) { return (size_t)s * 2 + m; }

__device__ inline float4* arena_base(const MapperDev& D, int s, int m, int active) {
  return D.arena + ((sm_index(s, m) * 2 + active) * (size_t)D.map_cap);
}
__device__ inline float4* carena_base(const MapperDev& D, int s, int m, int active) {
  return D.carena + ((sm_index(s, m) * 2 + active) * (size_t)D.map_cap);
}
__device__ inline uint2* ctab_base(const MapperDev& D, int s, int m, int active) {
  return D.ctab + ((sm_index(s, m) * 2 + active) * (size_t)D.map_cap * 4);
}
// lower corner of cube c (grid index) given the grid centre
__device__ inline void cube_corner(int c, const int* cen, int corner[3]) {
  corner[0] = ci_corner(c % CW, cen[0]);
  corner[1] = ci_corner((c / CW) % CH, cen[1]);
  corner[2] = ci_corner(c / (CW * CH), cen[2]);
}

// ---------------------------------------------------------------------------------------
// ring-buffer recentering (laser_mapping.cpp:252-444): content moves by shift[axis] cube
// indices, the slabs that wrap around are cleared.
// ---------------------------------------------------------------------------------------
// The fixed-point tokens move with their cubes (into tok_tmp, copied back on the same stream):
// a token left at the old index would send every moved cube through a full re-filter.
__global__ void k_shift_cubes(MapperDev D, const uint2* __restrict__ old_tab, uint2* new_tab, uint32_t* tok_tmp) {
  int s = D.s0 + blockIdx.y;
  const StreamFrame& F = D.fr[s];
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < 2 * NCUBE; t += gridDim.x * blockDim.x) {
    int m = t / NCUBE, c = t % NCUBE;
    int i = c % CW, j = (c / CW) % CH, k = c / (CW * CH);
    int oi = i - F.shift[0], oj = j - F.shift[1], ok = k - F.shift[2];
    uint2 v = make_uint2(0, 0);
    uint32_t tok = 0;
    if (oi >= 0 && oi < CW && oj >= 0 && oj < CH && ok >= 0 && ok < CD) {
      const size_t o = sm_index(s, m) * NCUBE + oi + CW * oj + CW * CH * ok;
      v = old_tab[o];
      tok = D.stable_tok[o];
    }
    new_tab[sm_index(s, m) * NCUBE + c] = v;
    tok_tmp[sm_index(s, m) * NCUBE + c] = tok;
  }
}

// PCL-order VoxelGrid (voxel_pcl.h) in a VX_THREADS workgroup owning the whole LDS: the sort's
// level lists in LDS (inputs up to ~115k points); the elements E and the stop lists A / B in LDS
// too for inputs up to MP_LDS_N points (the sort's dependent accesses are LDS latency, not L2),
// else at offset `so` of the (stream, map) sort scratch, where the sorted copy S always goes.
// Returns false (MAP_ERR_SORT) when the input is too large for the lists.
constexpr int MP_LDS_N = 8192;                                    // E 64 KiB + A, B 32 KiB each
constexpr int MP_LEV_W = 40;  // SsLevels words
static_assert(sizeof(SsLevels) <= 4 * MP_LEV_W, "SsLevels area");
constexpr int MP_SEG_LDS = (VX_LDS_WORDS - 256 - 2 * MP_LEV_W - 4 * MP_LDS_N) / 6;  // level lists beside them
static_assert(MP_SEG_LDS >= MP_LDS_N / (SS_THRESHOLD + 1) + 2, "level lists of an LDS-resident sort");
static_assert(VX_THREADS / 64 * SS_LOC_WORDS + 256 + 2 * MP_LEV_W <= VX_LDS_WORDS, "wave-local sort buffers");
// global-memory sorts: segments of at most MP_LDS_N elements are sorted whole in LDS
// (ss_sort_deferred: E, A, B and the level lists of one segment at a time)
constexpr int MP_DEF_SEG = MP_LDS_N / (SS_THRESHOLD + 1) + 2;
static_assert(4 * MP_LDS_N + 6 * MP_DEF_SEG + 256 + 2 * MP_LEV_W <= VX_LDS_WORDS, "deferred segment sort in LDS");
// sort scratch of a (stream, map): the stack at 0, the cubes' blocks of n + MP_SLACK from the
// frame's scratch_tail; the level lists and the deferred list of a global-memory sort at
// 9 (offset / 16) ints
constexpr uint32_t MP_SLACK = 64;
// cubes from 0, the stack (its own region: it may run beside the previous frame's re-filter)
// at mp_stack_offset
__host__ __device__ inline size_t mp_cube_scratch(const MapperDev& D) {
  return (size_t)D.scratch_cap + MP_SLACK * (INS_SLOTS + 1);
}
__host__ __device__ inline uint32_t mp_stack_offset(const MapperDev& D) { return (uint32_t)mp_cube_scratch(D); }
inline size_t mp_scratch(const MapperDev& D) { return mp_cube_scratch(D) + (size_t)D.max_in + MP_SLACK; }
template <typename PF>
__device__ inline bool map_voxel_pcl(const MapperDev& D, size_t sm, uint32_t so, const PF& P, int n, float leaf,
                                     const VxPclOut& O, uint32_t* lds, int* err) {
  const size_t ps = (size_t)D.scratch_cap + MP_SLACK * (INS_SLOTS + 1) + (size_t)D.max_in + MP_SLACK;
  const bool stk = so == mp_stack_offset(D);
  const size_t lim = stk ? ps : mp_cube_scratch(D);  // cubes stay below the stack
  if ((size_t)so + (uint32_t)n + MP_SLACK > lim) {
    if (threadIdx.x == 0) atomicOr(err, MAP_ERR_SORT);
    return false;
  }
  VxMisc& M = *reinterpret_cast<VxMisc*>(lds + VX_LDS_WORDS - 192);
  uint32_t* ws = lds + VX_LDS_WORDS - 256;
  SsLevels* lev = reinterpret_cast<SsLevels*>(lds + VX_LDS_WORDS - 256 - MP_LEV_W);
  const size_t b = sm * ps + so;
  if (n <= MP_LDS_N) {
    uint64_t* E = reinterpret_cast<uint64_t*>(lds);
    uint32_t* A = lds + 2 * MP_LDS_N;
    uint32_t* B = A + MP_LDS_N;
    int* seg0 = reinterpret_cast<int*>(B + MP_LDS_N);
    const VxPclScratch X{E, A, B, D.ps + b, lev, {seg0, seg0 + 3 * MP_SEG_LDS}, MP_SEG_LDS, nullptr,
                         D.pdbg ? (stk ? D.pdbg + 42 : D.pdbg + 11) : nullptr, D.pdbg ? (stk ? D.pdbg + 68 : D.pdbg + 66) : nullptr,
                         D.pdbg ? (stk ? D.pdbg + 65 : D.pdbg + 64) : nullptr};
    voxel_grid_pcl<VX_THREADS>(P, n, leaf, O, X, M, ws, err);
  } else {  // level lists in global memory; segments that fit the LDS are sorted there whole
    const int cap = (int)((n + MP_SLACK) / 16);
    int* seg0 = D.pseg + sm * (9 * (ps / 16) + 9) + 9 * (so / 16);
    const VxPclDefer dfr{MP_LDS_N,
                         seg0 + 6 * cap,
                         cap,
                         reinterpret_cast<uint64_t*>(lds),
                         lds + 2 * MP_LDS_N,
                         lds + 3 * MP_LDS_N,
                         reinterpret_cast<int*>(lds + 4 * MP_LDS_N),
                         reinterpret_cast<int*>(lds + 4 * MP_LDS_N) + 3 * MP_DEF_SEG,
                         MP_DEF_SEG,
                         reinterpret_cast<SsLevels*>(lds + VX_LDS_WORDS - 256 - 2 * MP_LEV_W)};
    const VxPclScratch X{D.pe + b, D.pa + b, D.pb + b, D.ps + b, lev, {seg0, seg0 + 3 * cap}, cap, lds,
                         D.pdbg ? (stk ? D.pdbg + 42 : D.pdbg + 11) : nullptr, D.pdbg ? (stk ? D.pdbg + 68 : D.pdbg + 66) : nullptr,
                         D.pdbg ? (stk ? D.pdbg + 65 : D.pdbg + 64) : nullptr};
    voxel_grid_pcl<VX_THREADS, true>(P, n, leaf, O, X, M, ws, err, &dfr);
  }
  return true;
}

// exact order (voxel_hot.h): the hot records of a filter of n points in the (stream, map) sort
// scratch at offset so (a block of n + MP_SLACK): rk in pa, fpos in pb, the member lists and the
// per-voxel records in pe (2 (n + MP_SLACK) words)
__device__ inline VxHot map_hot(const MapperDev& D, size_t sm, uint32_t so, uint32_t n) {
  const size_t b = sm * (mp_cube_scratch(D) + (size_t)D.max_in + MP_SLACK) + so;
  VxHot H;
  H.rk = D.pa + b;
  H.fpos = D.pb + b;
  H.hl = reinterpret_cast<uint32_t*>(D.pe + b);
  H.hv = H.hl + n;
  H.cap_h = n / 3 + 1;
  H.w = D.ps + b;  // (sorts of VH_MAX_N .. VH_BIG_N points: vh_sort_big)
  return H;
}

// ---------------------------------------------------------------------------------------
// VoxelGrid of the incoming feature clouds -> CornerStack / SurfStack (:492-500)
// ---------------------------------------------------------------------------------------
// one 1024-thread workgroup per (stream, map): grid B * 2
template <bool PCL>
__global__ void __launch_bounds__(VX_THREADS) k_stack_ds(MapperDev D) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[VX_LDS_WORDS];
  const int s = D.s0 + (blockIdx.x >> 1), m = blockIdx.x & 1;
  const StackIn& I = D.sin[s];
  if (!I.active) return;
  const size_t sm = sm_index(s, m);
  int* err = &D.stk_err[s];
  // PCL's order above VH_BIG_N points (or when vh_fixup cannot split the sort for the LDS): the
  // whole sort in global memory
  bool global = PCL && I.n[m] > VH_BIG_N;
  if (!global) {
  VoxSeg S;
  S.src1 = nullptr;
  S.tag1 = nullptr;
  S.n1 = 0;
  S.tag = 0;
  S.leaf = D.leaf[m];
  S.append_only = 0;
  S.tail = nullptr;
  S.res_off = nullptr;
  S.scratch_tail = nullptr;
  S.err = err;
  S.prof_seg = D.pdbg ? D.pdbg + 42 : nullptr;  // stack VoxelGrid phases: dbg[42..45]
  S.src0 = I.p[m];
  S.n0 = I.n[m];
  S.out = D.stack[m] + (size_t)s * D.max_in;
  S.cap = D.max_in;
  S.res_cnt = reinterpret_cast<uint32_t*>(&D.stk_n[2 * s + m]);
  S.scratch_pts = D.stk_pts + sm * D.max_in;
  S.scratch_idx = D.stk_idx + sm * D.max_in;
  S.scratch_cap = D.max_in;
  if (PCL) S.hot = map_hot(D, sm, mp_stack_offset(D), (uint32_t)I.n[m]);
  voxel_segment(S, lds);
  if (PCL) {  // PCL's summation order for the voxels of 3+ members (voxel_hot.h)
    const int he = vh_fixup<VX_THREADS>(VxSrc{I.p[m], I.n[m], nullptr}, I.n[m], S.out, S.hot, lds, VX_LDS_WORDS - 256,
                                        *reinterpret_cast<VxMisc*>(lds + VX_LDS_WORDS - 192), nullptr, err,
                                        D.pdbg ? D.pdbg + 54 : nullptr, D.pdbg ? D.pdbg + 77 : nullptr);
    global = he < 0;  // (over VH_MAX_N: the first partition left a part too large for the LDS)
    __syncthreads();
  }
  }
  if (PCL && global) {
    VxPclOut O;
    O.out = D.stack[m] + (size_t)s * D.max_in;
    O.cap = D.max_in;
    O.res_cnt = reinterpret_cast<uint32_t*>(&D.stk_n[2 * s + m]);
    map_voxel_pcl(D, sm, mp_stack_offset(D), VxPtrSrc{I.p[m]}, I.n[m], D.leaf[m], O, lds, err);
  }
}

// Few streams: the input-order stack VoxelGrid of a (stream, map) over stack_k workgroups.
// Every workgroup computes the same geometry and idx histogram (VX_NB buckets) from all the
// points, cuts the idx range into stack_k ranges of about equal point counts, and filters its
// own range (vx_group: hash, sorted unique voxels, member lists in input order, centroids) into
// the (stream, map) staging area at the point-count prefix of its range.  k_stack_cat then
// concatenates the ranges in idx order.  Same voxels, same member order, same sums: the bits of
// the one-workgroup filter.
constexpr int STACK_K_MAX = 16;
__global__ void __launch_bounds__(VX_THREADS) k_stack_part(MapperDev D) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[VX_LDS_WORDS];
  const int K = D.stack_k;
  const int j = blockIdx.x % K, pm = blockIdx.x / K;
  const int s = D.s0 + (pm >> 1), m = pm & 1;
  const StackIn& I = D.sin[s];
  if (!I.active) return;
  const size_t sm = sm_index(s, m);
  uint2* part = D.stk_part + sm * STACK_K_MAX;
  const uint32_t N = (uint32_t)I.n[m];
  const VxSrc P{I.p[m], (int)N, nullptr};
  float4* stage = D.stk_pts + sm * D.max_in;
  uint32_t* ws = lds + VX_LDS_WORDS - 256;
  VxMisc& M = *reinterpret_cast<VxMisc*>(lds + VX_LDS_WORDS - 192);
  const int tid = threadIdx.x;
  if (N == 0) {
    if (tid == 0) part[j] = make_uint2(0, 0);
    return;
  }
  unsigned long long tp = __builtin_readcyclecounter();  // phase counters (diagnostics)
  vx_geometry(P, N, D.leaf[m], M);
  vx_phase(D.pdbg ? D.pdbg + 42 : nullptr, 0, &tp);  // bounding box -> dbg[42] (summed over the K parts)
  const VxGeom g = M.g;
  if (g.overflow) {  // PCL: "Leaf size is too small" -> output = input (range 0 copies it)
    if (j == 0)
      for (uint32_t i = tid; i < N; i += VX_THREADS) stage[i] = P(i);
    if (tid == 0) part[j] = make_uint2(0, j == 0 ? N : 0u);
    return;
  }
  // idx histogram -> the ranges' bucket cuts by cumulative point count
  uint32_t* hist = lds + VX_HIST_WORD;
  // bucket(k) = floor(k mulc / 2^32) with mulc = floor(2^32 VX_NB / V): monotone in k and below
  // VX_NB for k < V, and a multiply instead of a 64-bit division per point (the histogram pass
  // spent most of its cycles in the division); blo(b) = ceil(b 2^32 / mulc) is its exact inverse
  // (the first key of bucket b), so the parts still cut the idx range at key boundaries
  const unsigned long long V = g.nvox;
  const unsigned long long mulc = (((unsigned long long)VX_NB) << 32) / V;
  auto bucket = [&](uint32_t k) { return (uint32_t)(((unsigned long long)k * mulc) >> 32); };
  auto blo = [&](uint32_t b) { return (uint32_t)((((unsigned long long)b << 32) + mulc - 1) / mulc); };
  for (int b = tid; b < VX_NB; b += VX_THREADS) hist[b] = 0;
  __syncthreads();
  // loads in flight together; the scan's points come in ring order, so a wave's lanes (consecutive
  // points) mostly fall in one bucket: each run of equal buckets adds its length with one LDS
  // atomic by its first lane (same-address atomics of a wave serialise).  Wave-uniform loop.
  {
    const int lane = tid & 63;
    const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    for (uint32_t ib = (uint32_t)(tid & ~63); ib < N; ib += VX_UNROLL * VX_THREADS) {
      uint32_t kk4[VX_UNROLL];
      vx_keys4(g, P, N, ib + lane, kk4);
#pragma unroll
      for (int u = 0; u < VX_UNROLL; ++u) {
        const uint32_t bk = kk4[u] != VX_EMPTY ? bucket(kk4[u]) : 0xFFFFFFFFu;
        const uint32_t prev = (uint32_t)__shfl_up((int)bk, 1, 64);
        const uint64_t starts = __ballot(lane == 0 || prev != bk);
        if (bk != 0xFFFFFFFFu && ((starts >> lane) & 1ull)) {
          const uint64_t after = starts & ~le;
          atomicAdd(&hist[bk], (uint32_t)((after ? __ffsll((long long)after) - 1 : 64) - lane));
        }
      }
    }
  }
  __syncthreads();
  // range r starts at the first bucket whose points-before count reaches r N / K: a block scan
  // of the histogram (two buckets per thread) and a test at every bucket
  static_assert(VX_NB == 2 * VX_THREADS, "two buckets per thread");
  const uint32_t h0 = hist[2 * tid], h1 = hist[2 * tid + 1];
  uint32_t tot;
  const uint32_t a0 = vx_block_scan(h0 + h1, ws, &tot), a1 = a0 + h0;  // points before buckets 2t, 2t+1
  const uint64_t thr0 = (uint64_t)j * N / K, thr1 = (uint64_t)(j + 1) * N / K;
  if (tid == 0) {
    M.sbase[0] = j == 0 ? 0u : (uint32_t)VX_NB;
    M.sbase[1] = j == K - 1 ? (uint32_t)VX_NB : (uint32_t)VX_NB;
    M.sfail = j == 0 ? 0 : (int)N;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t bb = 2 * tid + u, acc = u ? a1 : a0, prev = u ? a0 : a0 - (tid ? hist[2 * tid - 1] : 0u);
    const bool first = bb == 0;
    if (j > 0 && acc >= thr0 && (first || prev < thr0)) {
      M.sbase[0] = bb;
      M.sfail = (int)acc;
    }
    if (j < K - 1 && acc >= thr1 && (first || prev < thr1)) M.sbase[1] = bb;
  }
  __syncthreads();
  const uint32_t b0 = M.sbase[0], b1 = max(M.sbase[0], M.sbase[1]), base = (uint32_t)M.sfail;
  __syncthreads();  // vx_group reuses M
  vx_phase(D.pdbg ? D.pdbg + 91 : nullptr, 0, &tp);  // histogram + range cuts -> dbg[91]
  if (b0 >= b1) {  // empty range
    if (tid == 0) part[j] = make_uint2(base, 0);
    return;
  }
  VoxSeg S;
  S.src0 = I.p[m];
  S.n0 = (int)N;
  S.src1 = nullptr;
  S.tag1 = nullptr;
  S.n1 = 0;
  S.tag = 0;
  S.leaf = D.leaf[m];
  S.append_only = 0;
  S.out = stage;
  S.tail = nullptr;
  S.cap = (uint32_t)D.max_in;
  S.res_off = nullptr;
  S.res_cnt = nullptr;
  S.scratch_pts = nullptr;
  S.scratch_idx = D.stk_idx + sm * D.max_in;
  S.scratch_tail = nullptr;
  S.scratch_cap = (uint32_t)D.max_in;
  S.err = &D.stk_err[s];
  S.prof_seg = D.pdbg ? D.pdbg + 42 : nullptr;  // hash, sort + scan, members + centroids -> dbg[43..45]
  int moved = 0;
  const uint32_t klo = blo(b0), khi = b1 >= (uint32_t)VX_NB ? 0xFFFFFFFFu : blo(b1);
  const uint32_t U = vx_group(S, g, P, N, D.stk_idx + sm * D.max_in + base, klo, khi, base,
                              VX_LDS_WORDS - 256, lds, ws, M, &moved);
  if (tid == 0) {
    if (U == VX_OVERFLOW) atomicOr(&D.stk_err[s], MAP_ERR_STACK);
    part[j] = make_uint2(base, U == VX_OVERFLOW ? 0u : U);
  }
}

// the ranges of k_stack_part in idx order -> the stack and its count
__global__ void __launch_bounds__(VX_THREADS) k_stack_cat(MapperDev D) {
  const int s = D.s0 + (blockIdx.x >> 1), m = blockIdx.x & 1;
  if (!D.sin[s].active) return;
  const size_t sm = sm_index(s, m);
  const uint2* part = D.stk_part + sm * STACK_K_MAX;
  const float4* stage = D.stk_pts + sm * D.max_in;
  float4* out = D.stack[m] + (size_t)s * D.max_in;
  uint32_t o = 0;
  for (int j = 0; j < D.stack_k; ++j) {
    const uint2 pj = part[j];
    for (uint32_t i = threadIdx.x; i < pj.y; i += VX_THREADS) out[o + i] = stage[pj.x + i];
    o += pj.y;
  }
  if (threadIdx.x == 0) D.stk_n[2 * s + m] = (int)o;
}

// LaserMapping::input's initial guess (laser_mapping.cpp:206-207): pose = wmap (x) wodom
__host__ __device__ inline void pose_initial_guess(const double* wmap, const double* wodom, double* pose) {
  const dq qm{wmap[0], wmap[1], wmap[2], wmap[3]};
  const dq qo{wodom[0], wodom[1], wodom[2], wodom[3]};
  const dq q = qmul(qm, qo);
  const d3 r = qrot(qm, d3{wodom[4], wodom[5], wodom[6]});
  pose[0] = q.x; pose[1] = q.y; pose[2] = q.z; pose[3] = q.w;
  pose[4] = r.x + wmap[4];
  pose[5] = r.y + wmap[5];
  pose[6] = r.z + wmap[6];
}

// LaserMapping::transformUpdate (laser_mapping.cpp:147-151): wmap = pose (x) wodom^-1
__host__ __device__ inline void pose_transform_update(const double* pose, const double* wodom, double* wmap) {
  const dq qw{pose[0], pose[1], pose[2], pose[3]};
  const dq qo{wodom[0], wodom[1], wodom[2], wodom[3]};
  const dq qm = qmul(qw, qinv(qo));
  const d3 r = qrot(qm, d3{wodom[4], wodom[5], wodom[6]});
  wmap[0] = qm.x; wmap[1] = qm.y; wmap[2] = qm.z; wmap[3] = qm.w;
  wmap[4] = pose[4] - r.x;
  wmap[5] = pose[5] - r.y;
  wmap[6] = pose[6] - r.z;
}

// centerCube and the recentering count (laser_mapping.cpp:228-251): the window centre of a pose
// and how far the grid must shift (cen follows the shift); true if it shifts
__host__ __device__ inline bool frame_center(const double* pose, int* cen, int* center, int* shift) {
  const int dims[3] = {CW, CH, CD};
  bool any = false;
  for (int a = 0; a < 3; ++a) {
    int c = cube_of(pose[4 + a], cen[a]);
    shift[a] = 0;
    while (c < 3) { c++; cen[a]++; shift[a]++; }
    while (c >= dims[a] - 3) { c--; cen[a]--; shift[a]--; }
    center[a] = c;
    any |= shift[a] != 0;
  }
  return any;
}

// the window cubes (laserCloudValidInd, :455-472) and the cell-hash origin of F.center / F.cen
__host__ __device__ inline void frame_window(StreamFrame& F) {
  const int* c3 = F.center;
  int vn = 0;
  for (int i = c3[0] - 2; i <= c3[0] + 2; i++)
    for (int j = c3[1] - 2; j <= c3[1] + 2; j++)
      for (int k = c3[2] - 1; k <= c3[2] + 1; k++)
        if (i >= 0 && i < CW && j >= 0 && j < CH && k >= 0 && k < CD) F.window[vn++] = i + CW * j + CW * CH * k;
  F.valid_num = vn;
  // hash cell origin: world metres of the window's low corner, minus a 2-cell margin
  F.origin[0] = (c3[0] - 2 - F.cen[0]) * 50 - 25 - 2;
  F.origin[1] = (c3[1] - 2 - F.cen[1]) * 50 - 25 - 2;
  F.origin[2] = (c3[2] - 1 - F.cen[2]) * 50 - 25 - 2;
}

// per-frame resets of a stream record (the host's, or k_frame_prep's for a queued frame)
__host__ __device__ inline void frame_reset(StreamFrame& F) {
  F.shift[0] = F.shift[1] = F.shift[2] = 0;
  F.err = 0;
  F.nc_stack = F.ns_stack = 0;
  F.corner_num[0] = F.corner_num[1] = F.surf_num[0] = F.surf_num[1] = 0;
  F.sub_n[0] = F.sub_n[1] = 0;
  F.optimize = 0;
  F.cand[0] = F.cand[1] = 0;
}

// the frame's stack sizes and stack-filter errors into its stream records (after the stack
// kernels, which may have run while the previous frame was in flight)
// (agent-scope atomic loads: k_frame_prep reads them while other stacks of the same frame may
// still be running, and the words of all streams share lines that another stream's block of this
// XCD may have pulled into the L2 before this stack was written; an acquire fence instead would
// invalidate the XCD's whole L2 and cost the frame's later kernels their cached cubes)
__device__ inline void stack_counts(const MapperDev& D, int s, StreamFrame& F) {
  F.nc_stack = __hip_atomic_load(&D.stk_n[2 * s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  F.ns_stack = __hip_atomic_load(&D.stk_n[2 * s + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int e = __hip_atomic_load(&D.stk_err[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (e) {
    F.err |= e;
    __hip_atomic_store(&D.stk_err[s], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// after a stack launch on the stack stream: its number (agent scope); k_frame_prep
// waits for it on the device (a cross-stream event wait between two graph launches, pending when
// enqueued, costs ~5 us of the device's time, tools/mb_flush.hip)
__global__ void k_stack_done(unsigned long long* w, unsigned long long v) {
  // (the stack kernels before it on this stream ended with their own release: a relaxed store,
  // no L2 write-back here)
  if (threadIdx.x == 0) __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_stack_counts(MapperDev D) {
  const int s = D.s0 + blockIdx.x;
  StreamFrame& F = D.fr[s];
  if (threadIdx.x != 0 || !F.active) return;
  stack_counts(D, s, F);
}

// a queued frame's stream record, prepared on the device from what the frames before left (what
// the host does in mapper_enqueue): the initial guess (:206-207) with the transform of the
// stream's last solve, the window (:228-251, :455-472).  A frame that needs a recentering or an
// arena compaction, or follows a deferred one, is deferred: the stream stays inactive and the
// host runs it again on its own path (the device state is left as the frames before left it).
// All threads of the block: thread 0 decides from registers (one round of loads of the record),
// the window list is built one slot per thread (i, j, k order: :455-472).
__device__ inline void frame_prep_device(const MapperDev& D, StreamFrame& F, const FrameIn& I) {
  __shared__ int ok, c3s[3], cens[3];
  __shared__ uint64_t vmask[2];
  const int tid = threadIdx.x;
  if (tid == 0) {
    const int prev_deferred = F.deferred;
    double wmap[7];
    for (int i = 0; i < 7; ++i) wmap[i] = F.wmap[i];
    int cen[3] = {F.cen[0], F.cen[1], F.cen[2]};
    const uint32_t t0 = F.arena_tail[0], t1 = F.arena_tail[1];
    F.active = 0;
    ok = 0;
    if (I.active) {
      double pose[7];
      pose_initial_guess(wmap, I.wodom, pose);
      int center[3], shift[3];
      const bool shifted = frame_center(pose, cen, center, shift);
      const bool compact = t0 > D.compact_at || t1 > D.compact_at;
      const bool forced = D.defer_every > 0 && I.epoch % (uint32_t)D.defer_every == 0;
      for (int i = 0; i < 7; ++i) F.wodom[i] = I.wodom[i];
      if (prev_deferred || shifted || compact || forced) {
        F.deferred = 1;
      } else {
        frame_reset(F);
        F.active = 1;
        for (int i = 0; i < 7; ++i) F.pose[i] = pose[i];
        for (int a = 0; a < 3; ++a) {
          F.center[a] = c3s[a] = center[a];
          cens[a] = cen[a];
        }
        F.origin[0] = (center[0] - 2 - cen[0]) * 50 - 25 - 2;  // as frame_window
        F.origin[1] = (center[1] - 2 - cen[1]) * 50 - 25 - 2;
        F.origin[2] = (center[2] - 1 - cen[2]) * 50 - 25 - 2;
        F.epoch = I.epoch;
        F.in_ptr[0] = I.in_ptr[0];
        F.in_ptr[1] = I.in_ptr[1];
        F.nc_in = I.n[0];
        F.ns_in = I.n[1];
        ok = 1;
      }
    }
  }
  __syncthreads();
  if (!ok) return;
  // window slot t = (i * 5 + j) * 3 + k of the 5 x 5 x 3 cubes around the centre, kept if inside
  // the grid, in that order (frame_window)
  const int t = tid;
  const int i = c3s[0] - 2 + t / 15, j = c3s[1] - 2 + (t / 3) % 5, k = c3s[2] - 1 + t % 3;
  const bool in = t < 75 && i >= 0 && i < CW && j >= 0 && j < CH && k >= 0 && k < CD;
  const uint64_t b = __ballot(in);
  const int w = tid >> 6, lane = tid & 63;
  if (lane == 0 && w < 2) vmask[w] = b;
  __syncthreads();
  const int pos = (w == 1 ? __popcll(vmask[0]) : 0) + __popcll(b & ((1ull << lane) - 1));
  if (in) F.window[pos] = i + CW * j + CW * CH * k;
  if (tid == 0) F.valid_num = __popcll(vmask[0]) + __popcll(vmask[1]);
  __syncthreads();
}

// the graph path's last kernel: every stream record to page-locked host memory (write-through
// stores), then the frame's number (FrameIn.epoch) to the host's done word: the host waits on
// that word instead of an event record and a D2H copy between frames
__global__ void __launch_bounds__(256) k_frame_out(MapperDev D, StreamFrame* out, unsigned long long* done) {
  constexpr int W = (int)(sizeof(StreamFrame) / 8);
  static_assert(sizeof(StreamFrame) % 8 == 0, "record copy granularity");
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(D.fr + D.s0);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(out);
  for (int w = threadIdx.x; w < D.B * W; w += blockDim.x)
    __hip_atomic_store(dst + w, src[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // every lane's write-through stores complete before the done word (no fence: a system-scope
  // release writes back the whole L2, dirty with the frame's map; ~5 us, tools/mb_flush.hip)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long e = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(&D.fin[0].epoch),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & 0xFFFFFFFFull;
    __hip_atomic_store(done, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}


// FrameIn from page-locked host memory into LDS: one system-scope load per lane, all in flight
// together (the host wrote it before the launch; each read crosses the host link)
constexpr int FRAME_IN_WORDS = (int)(sizeof(FrameIn) / 8);
static_assert(sizeof(FrameIn) % 8 == 0 && FRAME_IN_WORDS <= 64, "FrameIn copy granularity");
__device__ inline void load_frame_in(const FrameIn* p, FrameIn* lds) {
  const int w = threadIdx.x;
  if (w < FRAME_IN_WORDS)
    reinterpret_cast<unsigned long long*>(lds)[w] =
        __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p) + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---------------------------------------------------------------------------------------
// submap: offsets of the window cubes (laserCloudCornerFromMap concatenation order)
// ---------------------------------------------------------------------------------------
__device__ inline void submap_prep(const MapperDev& D, int s, StreamFrame& F) {
  // one wave per map; window slots 2*lane, 2*lane+1 (valid_num <= 75 <= 128)
  const int m = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint2* tab = D.cube_tab + sm_index(s, m) * NCUBE;
  const int vn = F.valid_num;
  const int w0 = 2 * lane, w1 = 2 * lane + 1;
  const uint32_t* wc = D.wcnt + sm_index(s, m) * WIN_MAX;  // sharded: summed over the ranks
  const uint32_t c0 = w0 < vn ? (D.sharded ? wc[w0] : tab[F.window[w0]].y) : 0u;
  const uint32_t c1 = w1 < vn ? (D.sharded ? wc[w1] : tab[F.window[w1]].y) : 0u;
  const uint32_t inc = wave_incl_scan_u(c0 + c1);
  uint32_t total = __shfl(inc, 63, 64);
  const bool over = total > (uint32_t)D.sub_cap;
  const uint32_t ex = over ? 0u : inc - (c0 + c1);
  if (w0 < vn) F.sub_off[m][w0] = ex;
  if (w1 < vn) F.sub_off[m][w1] = over ? 0u : ex + c0;
  if (lane == 0) {
    if (over) {
      atomicOr(&F.err, MAP_ERR_SUBMAP);
      total = 0;
    }
    F.sub_off[m][vn] = total;
    F.sub_n[m] = total;
    F.scratch_tail[m] = 0;  // re-VoxelGrid scratch (bounded by max_submap_points + stacks)
    F.hot_tail[m] = 0;
    F.extra_n[m] = 0;
    if (m == 0) F.vx_bytes = 0;
  }
  __syncthreads();
  // laser_mapping.cpp:514
  if (threadIdx.x == 0) F.optimize = (F.sub_n[0] > 10 && F.sub_n[1] > 50) ? 1 : 0;
}

__global__ void __launch_bounds__(128) k_submap_prep(MapperDev D) {
  const int s = D.s0 + blockIdx.x;
  StreamFrame& F = D.fr[s];
  if (blockIdx.x == 0 && threadIdx.x < RQ_CLASSES) D.rq_ctl[threadIdx.x] = 0u;  // this frame's k_revox list
  if (!F.active) return;
  submap_prep(D, s, F);
}

// the graph path's first kernel: a queued frame's records (frame_prep_device), the stack sizes
// (k_stack_counts) and the submap offsets (k_submap_prep) in one launch
__global__ void __launch_bounds__(128) k_frame_prep(MapperDev D) {
  const int s = D.s0 + blockIdx.x;
  StreamFrame& F = D.fr[s];
  if (blockIdx.x == 0 && threadIdx.x < RQ_CLASSES) D.rq_ctl[threadIdx.x] = 0u;  // this frame's k_revox list
  __shared__ int go;
  __shared__ FrameIn I;
  const unsigned long long t0 = __builtin_readcyclecounter();
  load_frame_in(D.fin + s, &I);
  __syncthreads();
  if (threadIdx.x == 0 && I.active && I.stack_seq) {  // the stream's stacks (launched on the stack stream)
    uint32_t spins = 0;
    while (__hip_atomic_load(D.stk_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < I.stack_seq) {
      if (++spins > (1u << 24)) {
        atomicOr(&F.err, MAP_ERR_STACK_WAIT);
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    // the stack sizes are read with agent-scope loads (stack_counts); the stack points only by
    // later kernels, which start after every stack of the frame has ended
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (I.mode == 1) frame_prep_device(D, F, I);  // (block-uniform branch)
  const unsigned long long t2 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) {
    if (F.active) stack_counts(D, s, F);
    go = F.active;
  }
  __syncthreads();
  if (!go) return;
  const unsigned long long t3 = __builtin_readcyclecounter();
  submap_prep(D, s, F);
  if (D.pdbg && threadIdx.x == 0) {  // cycles: [58] FrameIn load, [59] device prep, [60] stack counts, [61] submap
    const unsigned long long t4 = __builtin_readcyclecounter();
    atomicAdd(&D.pdbg[58], t1 - t0);
    atomicAdd(&D.pdbg[59], t2 - t1);
    atomicAdd(&D.pdbg[60], t3 - t2);
    atomicAdd(&D.pdbg[61], t4 - t3);
    atomicAdd(&D.pdbg[62], 1ull);
    if (I.mode == 1) atomicAdd(&D.pdbg[63], 1ull);  // frames prepared on the device
  }
}

// sharded: this rank's point count of every window cube, all-reduced before k_submap_prep so
// that every rank sees the whole submap's sizes and concatenation offsets (:475-489, :514)
__global__ void __launch_bounds__(256) k_submap_count(MapperDev D) {
  const int s = D.s0 + blockIdx.x;
  const StreamFrame& F = D.fr[s];
  for (int t = threadIdx.x; t < 2 * WIN_MAX; t += blockDim.x) {
    const int m = t / WIN_MAX, w = t % WIN_MAX;
    uint32_t c = 0;
    if (F.active && w < F.valid_num) c = D.cube_tab[sm_index(s, m) * NCUBE + F.window[w]].y;
    D.wcnt[sm_index(s, m) * WIN_MAX + w] = c;
  }
}

// ---------------------------------------------------------------------------------------
// correspondences of one outer round (laser_mapping.cpp:545-699) -> factor records
// ---------------------------------------------------------------------------------------
// pass 1: exact 5-NN of every query (laser_mapping.cpp:554, :633; accepted only if the 5th is
// within 1 m: :557, :642) over the window cubes' cell indexes (cubeindex.h).  Distances are
// FLANN's L2_Simple<float>; ties go to the lower submap index (sub_off[slot] + position in
// the cube).  Output: positions of the 5 neighbours in the cell-sorted arena, -1: none.
struct Near5 {
  float d[5];
  int id[5];   // submap index (tie-break)
  int pos[5];  // cell-sorted arena position
};
__device__ inline void near5_offer(Near5& T, float d, int id, int pos) {
  if (!(d < T.d[4] || (d == T.d[4] && id < T.id[4]))) return;
  T.d[4] = d; T.id[4] = id; T.pos[4] = pos;
#pragma unroll
  for (int k = 4; k > 0; --k) {
    if (T.d[k] < T.d[k - 1] || (T.d[k] == T.d[k - 1] && T.id[k] < T.id[k - 1])) {
      float td = T.d[k]; T.d[k] = T.d[k - 1]; T.d[k - 1] = td;
      int ti = T.id[k]; T.id[k] = T.id[k - 1]; T.id[k - 1] = ti;
      int tp = T.pos[k]; T.pos[k] = T.pos[k - 1]; T.pos[k - 1] = tp;
    }
  }
}
__device__ inline int floor_div50(int v) { return v >= 0 ? v / 50 : -((-v + 49) / 50); }

struct WinMap {  // per (stream, map) window cubes, in LDS
  uint32_t off[WIN_MAX], n[WIN_MAX], tsize[WIN_MAX];
  int sub[WIN_MAX];
};

// L lanes per query (L | 64): the lanes of a group visit the same cells and split each cell's
// points; the pruning bound is the group minimum of the lanes' 5th distances (each bounds the
// union's 5th from above, so it is safe), and a butterfly merge leaves the union's 5 nearest in
// every lane.  The result is the L = 1 result (the minimum over (d, key) of the same
// candidates); L > 1 shortens each query's chain of dependent loads.
// block -> (stream, member): stream b % B, member b / B (a stream's blocks on one XCD, b % 8,
// when B is a multiple of 8: they share that XCD's L2 copy of the stream's cell indexes)
__device__ inline void corr_block(const MapperDev& D, int* s, int* blk) {
  *s = D.s0 + blockIdx.x % D.B;
  *blk = blockIdx.x / D.B;
}

#ifndef KNN_WAVES
#define KNN_WAVES 7  // 72 VGPRs, 20 B spill outside the cell loop: 6 -> 7 waves, correspondence -8%
#endif
// CS (cell split): the L lanes of a query take different cells, lane g the cells g, g + L, ...
// of the nearest-first order, each scanning all of its cell's points, with the group minimum of
// their 5th distances as the shared pruning bound: a query's chain of dependent probes is 27 / L
// steps long instead of 27 (few streams leave the chip mostly idle: latency, not issue, bounds
// the search).  Without CS the lanes share each cell and split its points.
template <int L, bool CS = false>
__global__ void __launch_bounds__(CORR_THREADS) __attribute__((amdgpu_waves_per_eu(CS ? 4 : KNN_WAVES, 8))) k_knn(MapperDev D, int round) {
  __shared__ WinMap W[2];
  __shared__ int slot_of[75];  // 5 x 5 x 3 window position -> slot (laserCloudValidInd order)
  int s, blk;
  corr_block(D, &s, &blk);
  StreamFrame& F = D.fr[s];
  if (!F.active) return;
  double X[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) X[i] = F.pose[i];
  if (blk == 0 && threadIdx.x < LM_SYNC_WORDS) D.lm_sync[((size_t)s * 2 + round) * LM_SYNC_WORDS + threadIdx.x] = 0;
  if (blk == 0 && threadIdx.x == 0) lm_init(F.lm[round], X, 4, F.optimize != 0);
  if (!F.optimize) return;  // k_geom types every record 0
  const int tid = threadIdx.x;
  const int c0 = F.center[0] - 2, c1 = F.center[1] - 2, c2 = F.center[2] - 1;
  if (tid < 75) slot_of[tid] = -1;
  __syncthreads();
  if (tid < F.valid_num) {
    const int cube = F.window[tid];
    const int ci = cube % CW, cj = (cube / CW) % CH, ck = cube / (CW * CH);
    slot_of[(ci - c0) * 15 + (cj - c1) * 3 + (ck - c2)] = tid;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const uint2 cv = D.cube_tab[sm_index(s, m) * NCUBE + cube];
      W[m].off[tid] = cv.x;
      W[m].n[tid] = cv.y;
      W[m].tsize[tid] = cv.y ? ci_table_size(cv.y) : 0u;
      W[m].sub[tid] = F.sub_off[m][tid];
    }
  }
  __syncthreads();
  const int nc = F.nc_stack, ns = F.ns_stack;
  const size_t rb = (size_t)s * 2 * D.max_in;
  uint32_t ncand = 0;
  const int gsub = tid % L;
  const int nblk = CS ? D.knn_blk : CORR_BLK;
  for (int ridx = blk * (CORR_THREADS / L) + tid / L; ridx < nc + ns; ridx += nblk * (CORR_THREADS / L)) {
    const int m = ridx < nc ? 0 : 1;  // corners [0, nc), surfs [nc, nc + ns)
    const int qi = m == 0 ? ridx : ridx - nc;
    const float4 q = to_map(X, D.stack[m][(size_t)s * D.max_in + qi]);
    const float4* cp = carena_base(D, s, m, F.arena_active[m]);
    const uint2* ct = ctab_base(D, s, m, F.arena_active[m]);
    const WinMap& WM = W[m];
    Near5 T;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      T.d[k] = INFINITY;
      T.id[k] = 0x7FFFFFFF;
      T.pos[k] = -1;
    }
    const float fx = floorf(q.x), fy = floorf(q.y), fz = floorf(q.z);
    const int qx = (int)fx, qy = (int)fy, qz = (int)fz;
    const float lx = q.x - fx, hx = (fx + 1.0f) - q.x;
    const float ly = q.y - fy, hy = (fy + 1.0f) - q.y;
    const float lz = q.z - fz, hz = (fz + 1.0f) - q.z;
    // points of cell (x, y, z) filed in cube (bi, bj, bk) at local (ax, ay, az)
    auto scan = [&](int bi, int bj, int bk, int ax, int ay, int az) {
      const int wx = bi - c0, wy = bj - c1, wz = bk - c2;
      if (wx < 0 || wx > 4 || wy < 0 || wy > 4 || wz < 0 || wz > 2) return;  // not in the submap
      const int sl = slot_of[wx * 15 + wy * 3 + wz];
      if (sl < 0) return;
      const uint32_t n = WM.n[sl];
      if (n == 0) return;
      const uint32_t off = WM.off[sl];
      const uint2 e = ci_find(ct + 4 * (size_t)off, WM.tsize[sl],
                              (uint32_t)ax | ((uint32_t)ay << 6) | ((uint32_t)az << 12));
      ncand += e.y;
      const int sub = WM.sub[sl];
      for (uint32_t k = CS ? 0 : gsub; k < e.y; k += CS ? 1 : L) {
        const uint32_t pos = off + e.x + k;
        const float4 p = cp[pos];
        // sharded: submap position x ranks + rank keeps the key unique (and equal to the
        // unsharded key at one rank)
        const int key = (sub + __float_as_int(p.w)) * D.nrank + D.rank;
        near5_offer(T, fdist2(q.x, q.y, q.z, p.x, p.y, p.z), key, (int)pos);
      }
    };
    for (int ob = 0; ob < 27; ob += CS ? L : 1) {
      const int o = CS ? ob + gsub : ob;
      const uint32_t code = cell_order_code(o < 27 ? o : 0);
      const int dx = (int)(code & 3u) - 1, dy = (int)((code >> 2) & 3u) - 1, dz = (int)(code >> 4) - 1;
      const float gx = dx < 0 ? lx : (dx > 0 ? hx : 0.f);
      const float gy = dy < 0 ? ly : (dy > 0 ? hy : 0.f);
      const float gz = dz < 0 ? lz : (dz > 0 ? hz : 0.f);
      float bound = fminf(T.d[4], 1.0f) * 1.01f + 1e-6f;  // rounding margin
#pragma unroll
      for (int o2 = 1; o2 < L; o2 <<= 1) bound = fminf(bound, __shfl_xor(bound, o2, 64));
      if (o >= 27 || gx * gx + gy * gy + gz * gz > bound) continue;
      const int x = qx + dx, y = qy + dy, z = qz + dz;
      const int bi = floor_div50(x + 25) + F.cen[0], bj = floor_div50(y + 25) + F.cen[1],
                bk = floor_div50(z + 25) + F.cen[2];
      int cx[3] = {bi, bj, bk};
      int lc[3];
      const int cv[3] = {x, y, z};
#pragma unroll
      for (int a = 0; a < 3; ++a) lc[a] = cv[a] - ci_corner(cx[a], F.cen[a]);
      scan(bi, bj, bk, lc[0], lc[1], lc[2]);
      // the reference files points at an exact negative multiple of 50 (v + 25) in the cube
      // below (laser_mapping.cpp:747-756): local coordinate 50 there
      int edge = 0;
#pragma unroll
      for (int a = 0; a < 3; ++a)
        if (cv[a] + 25 < 0 && (cv[a] + 25) % 50 == 0) edge |= 1 << a;
      for (int e = edge; e; e = (e - 1) & edge) {
        int b2[3], l2[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          b2[a] = (e >> a) & 1 ? cx[a] - 1 : cx[a];
          l2[a] = (e >> a) & 1 ? 50 : lc[a];
        }
        scan(b2[0], b2[1], b2[2], l2[0], l2[1], l2[2]);
      }
    }
#pragma unroll
    for (int o = 1; o < L; o <<= 1) {  // butterfly: disjoint candidate sets at every step
      float pd[5];
      int pid[5], ppos[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        pd[k] = __shfl_xor(T.d[k], o, 64);
        pid[k] = __shfl_xor(T.id[k], o, 64);
        ppos[k] = __shfl_xor(T.pos[k], o, 64);
      }
#pragma unroll
      for (int k = 0; k < 5; ++k)
        if (ppos[k] >= 0) near5_offer(T, pd[k], pid[k], ppos[k]);
    }
    if (gsub != 0) continue;
    if (D.sharded) {  // this rank's candidates; the 1 m test follows the merge (k_nn_merge)
      NnRec& o = D.nn_send[D.q_off[s] + ridx];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        o.d[k] = T.d[k];
        o.id[k] = T.id[k];
        const float4 p = T.pos[k] >= 0 ? cp[T.pos[k]] : make_float4(0.f, 0.f, 0.f, 0.f);
        o.x[k] = p.x;
        o.y[k] = p.y;
        o.z[k] = p.z;
      }
      continue;
    }
    const bool ok = T.d[4] < 1.0f;
#pragma unroll
    for (int k = 0; k < 5; ++k) D.knn_id[k * D.knn_stride + rb + ridx] = ok ? T.pos[k] : -1;
  }
  unsigned long long wc = ncand;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) wc += __shfl_xor(wc, o, 64);
  if ((threadIdx.x & 63) == 0 && wc) atomicAdd(&F.cand[round], wc);
}

// sharded: merge every rank's 5 candidates into the exact 5-NN of the whole submap (each
// rank's list is exact over its own points, so the union's 5 smallest (d, key) are the
// unsharded result), then the 1 m acceptance (:557, :642).  Neighbours go to nn_xyz.
__global__ void __launch_bounds__(CORR_THREADS) k_nn_merge(MapperDev D) {
  const int s = D.s0 + blockIdx.x % D.B, blk = blockIdx.x / D.B;
  const StreamFrame& F = D.fr[s];
  if (!F.active || !F.optimize) return;
  const int nq = F.nc_stack + F.ns_stack;
  const size_t rb = (size_t)s * 2 * D.max_in;
  const size_t qtot = (size_t)D.q_off[D.s0 + D.B];  // records per rank
  for (int ridx = blk * CORR_THREADS + threadIdx.x; ridx < nq; ridx += CORR_BLK * CORR_THREADS) {
    Near5 T;
    float px[5], py[5], pz[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      T.d[k] = INFINITY;
      T.id[k] = 0x7FFFFFFF;
      T.pos[k] = -1;
      px[k] = py[k] = pz[k] = 0.f;
    }
    for (int r = 0; r < D.nrank; ++r) {
      const NnRec& c = D.nn_recv[(size_t)r * qtot + D.q_off[s] + ridx];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const float d = c.d[k];
        const int id = c.id[k];
        if (!(d < T.d[4] || (d == T.d[4] && id < T.id[4]))) break;  // c is sorted
        // insert at the tail, bubble up; pos carries the candidate's slot in (px, py, pz)
        int j = 4;
        while (j > 0 && (d < T.d[j - 1] || (d == T.d[j - 1] && id < T.id[j - 1]))) {
          T.d[j] = T.d[j - 1];
          T.id[j] = T.id[j - 1];
          px[j] = px[j - 1];
          py[j] = py[j - 1];
          pz[j] = pz[j - 1];
          --j;
        }
        T.d[j] = d;
        T.id[j] = id;
        px[j] = c.x[k];
        py[j] = c.y[k];
        pz[j] = c.z[k];
      }
    }
    const bool ok = T.d[4] < 1.0f;
    D.knn_id[rb + ridx] = ok ? 0 : -1;
    if (ok) {
#pragma unroll
      for (int k = 0; k < 5; ++k) D.nn_xyz[k * D.knn_stride + rb + ridx] = make_float4(px[k], py[k], pz[k], 0.f);
    }
  }
}

// pass 2: line PCA / plane fit of the 5 neighbours -> factor records (laser_mapping.cpp:557-603,
// :642-680)
__global__ void __launch_bounds__(CORR_THREADS) k_geom(MapperDev D, int round) {
  int s, blk;
  corr_block(D, &s, &blk);
  StreamFrame& F = D.fr[s];
  if (!F.active) return;
  const int nc = F.nc_stack, ns = F.ns_stack;
  const size_t rb = (size_t)s * 2 * D.max_in;
  uint32_t n_edge = 0, n_plane = 0;  // reduced once per wave after the loop
  for (int ridx = blk * CORR_THREADS + threadIdx.x; ridx < nc + ns; ridx += CORR_BLK * CORR_THREADS) {
    if (!F.optimize) {
      D.r_type[rb + ridx] = 0;
      continue;
    }
    const int m = ridx < nc ? 0 : 1;
    const int qi = m == 0 ? ridx : ridx - nc;
    const float4 po = D.stack[m][(size_t)s * D.max_in + qi];
    int type = 0;
    double a[3] = {0, 0, 0}, b[3] = {0, 0, 0};
    if (D.knn_id[rb + ridx] >= 0) {
      const float4* lin = carena_base(D, s, m, F.arena_active[m]);
      float nb[5][3];
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        const float4 p = D.sharded ? D.nn_xyz[j * D.knn_stride + rb + ridx] : lin[D.knn_id[j * D.knn_stride + rb + ridx]];
        nb[j][0] = p.x;
        nb[j][1] = p.y;
        nb[j][2] = p.z;
      }
      if (m == 0) {
        d3 pa, pb;
        if (edge_from_nbrs(nb, pa, pb)) {
          type = 1;
          d3 de{pa.x - pb.x, pa.y - pb.y, pa.z - pb.z};
          double dn = sqrt(de.x * de.x + de.y * de.y + de.z * de.z);
          a[0] = pa.x; a[1] = pa.y; a[2] = pa.z;
          b[0] = de.x / dn; b[1] = de.y / dn; b[2] = de.z / dn;
          ++n_edge;
        }
      } else {
        d3 n;
        double d;
        if (plane_from_nbrs(nb, n, d)) {
          type = 3;
          a[0] = n.x; a[1] = n.y; a[2] = n.z;
          b[0] = d;
          ++n_plane;
        }
      }
    }
    D.r_type[rb + ridx] = type;
    D.r_px[rb + ridx] = po.x;
    D.r_py[rb + ridx] = po.y;
    D.r_pz[rb + ridx] = po.z;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      D.r_a[k][rb + ridx] = a[k];
      D.r_b[k][rb + ridx] = b[k];
    }
  }
  uint32_t we = n_edge, wp = n_plane;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    we += __shfl_xor(we, o, 64);
    wp += __shfl_xor(wp, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (we) atomicAdd(&F.corner_num[round], (int)we);
    if (wp) atomicAdd(&F.surf_num[round], (int)wp);
  }
}

// LM evaluation pass at the state's evaluation point (lm.h)
// reduce: sharded over several ranks, the stream's last workgroup to finish also sums the
// stream's partials in a fixed order into lm_red[s] (then all-reduced over the ranks): plain
// partial stores + agent-scope release + a ticket; the last acquires before it reads
__global__ void __launch_bounds__(LM_THREADS) k_lm_eval(MapperDev D, int round, int reduce) {
  const int s = D.s0 + blockIdx.x / LM_EBLK, blk = blockIdx.x % LM_EBLK;
  const StreamFrame& F = D.fr[s];
  if (!F.active) return;
  const size_t rb = (size_t)s * 2 * D.max_in;
  const LmRecView R{D.r_type + rb, D.r_px + rb, D.r_py + rb, D.r_pz + rb, D.r_a[0] + rb,
                    D.r_a[1] + rb, D.r_a[2] + rb, D.r_b[0] + rb, D.r_b[1] + rb, D.r_b[2] + rb};
  // sharded: this rank's workgroups are blocks rank * LM_EBLK + blk of nrank * LM_EBLK
  lm_eval_block<LM_THREADS>(R, F.nc_stack + F.ns_stack, F.lm[round], D.rank * LM_EBLK + blk, D.nrank * LM_EBLK,
                            D.partials + ((size_t)s * LM_EBLK + blk) * LM_NACC);
  if (!reduce || F.lm[round].status == LM_DONE) return;  // (uniform over the stream's workgroups)
  __shared__ int last;
  __syncthreads();  // this workgroup's partial stored
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const uint32_t t = __hip_atomic_fetch_add(&D.lm_tick[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == (uint32_t)LM_EBLK - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(&D.lm_tick[s], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x < 64) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (every reading wave)
  if (threadIdx.x < LM_NACC) {
    const double* p = D.partials + (size_t)s * LM_EBLK * LM_NACC;
    double v = 0.0;
    for (int c = 0; c < LM_EBLK; ++c) v += p[(size_t)c * LM_NACC + threadIdx.x];
    D.lm_red[(size_t)s * LM_NACC + threadIdx.x] = v;
  }
}

// LM step: one wave per stream; on termination the best point becomes the stream pose
// (Ceres writes it back into the parameter blocks, laser_mapping.cpp:535-536)
__global__ void __launch_bounds__(64) k_lm_step(MapperDev D, int round) {
  const int s = D.s0 + blockIdx.x;
  StreamFrame& F = D.fr[s];
  if (!F.active) return;
  LmState& S = F.lm[round];
  if (D.sharded)  // the all-reduced sums: every rank takes the identical step
    lm_step_wave(D.lm_red + (size_t)s * LM_NACC, 1, S, F.pose);
  else
    lm_step_wave(D.partials + (size_t)s * LM_EBLK * LM_NACC, LM_EBLK, S, F.pose);  // pose = best when done
}

// ---------------------------------------------------------------------------------------
// One launch per outer round: all <= 5 LM passes of every stream.  G workgroups per stream
// evaluate a share of the records each; the stream's leader (g = 0) keeps the trust-region
// state in its LDS, reduces the workers' partials and runs the step.  Hand-offs follow the
// agent-scope release/acquire recipe (cdna_hip_programming.md §6 Guideline 16): partials are
// plain stores + drain + release fence + relaxed ticket; the eval point is published with sc1
// (atomic) stores + drain + a relaxed flag; every consumer polls relaxed and acquires once.
// Shares are claimed per pass by whichever workgroups run (no residency needed), and every spin is
// bounded (MAP_ERR_LM_SYNC, the stream's LM then stops).
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(LM_THREADS) k_lm_round(MapperDev D, int round, int G) {
  // block b -> stream b % Bp, member b / Bp with B padded to a multiple of 8 (the padding
  // blocks leave at once): all of a stream's blocks share an XCD (b % 8), so its hand-offs
  // stay in one L2 (placement is speed only)
  const int Bp = lm_padded(D.B), sl = blockIdx.x % Bp, g = blockIdx.x / Bp;
  if (sl >= D.B) return;
  const int s = D.s0 + sl;
  StreamFrame& F = D.fr[s];
  if (!F.active) return;
  const size_t rb = (size_t)s * 2 * D.max_in;
  LmJob J;
  J.S = &F.lm[round];
  J.R = LmRecView{D.r_type + rb, D.r_px + rb, D.r_py + rb, D.r_pz + rb, D.r_a[0] + rb, D.r_a[1] + rb,
                  D.r_a[2] + rb, D.r_b[0] + rb, D.r_b[1] + rb, D.r_b[2] + rb};
  J.nrec = F.nc_stack + F.ns_stack;
  J.part = D.partials + (size_t)s * D.max_chunks * LM_NACC;
  J.sync = D.lm_sync + ((size_t)s * 2 + round) * LM_SYNC_WORDS;
  J.xpub = D.lm_xpub + ((size_t)s * 2 + round) * 8;
  J.best_out = F.pose;
  J.err = &F.err;
  J.err_code = MAP_ERR_LM_SYNC;
  J.prof = D.pdbg ? D.pdbg + 17 : nullptr;
  if (D.ipc_tab) {  // ranks in other processes: the per-pass sums meet in their mapped buffers
    J.rank = D.rank;
    J.nrank = D.nrank;
    J.ipc = D.ipc_tab;
    J.ipc_slot_off = (((size_t)(F.epoch & 1u) * D.ipc_B + s) * 2 + round) * LM_MAX_PASSES * LM_NACC;
    J.ipc_flag_off = (size_t)s * 2 + round;
    J.flag_base = F.epoch * (uint32_t)LM_MAX_PASSES;
  }
  lm_round_device<LM_THREADS>(J, g, G);
}

// The LM round of every rank of an in-process sharded group in ONE launch (comm_group_launch):
// the ranks' leaders wait for each other's per-pass sums (peer slots, lm.h), which separate
// launches could not do safely (two streams' kernels may share a hardware queue, one behind the
// other).  What k_lm_round reads of each rank's MapperDev:
struct LmRankArgs {
  StreamFrame* fr;
  const int* r_type;
  const float *r_px, *r_py, *r_pz;
  const double* r_a[3];
  const double* r_b[3];
  double* partials;
  uint32_t* lm_sync;
  double* lm_xpub;
  unsigned long long* pdbg;
  int max_in, max_chunks, B, s0;
};
struct LmGroupArgs {
  LmRankArgs r[LOAM_LOCAL_MAX_RANKS];
  double* peer;        // MapperDev::lm_peer (the group's)
  uint32_t* peer_flag;
  int nrank;
};
// blocks: the R x Bp leaders first (rank-major, so every leader is dispatched before any member),
// then each rank's members; a stream's blocks are congruent mod 8 (one XCD) as in k_lm_round
__global__ void __launch_bounds__(LM_THREADS) k_lm_group(LmGroupArgs A, int round, int G) {
  const int R = A.nrank, Bp = lm_padded(A.r[0].B);
  int b = blockIdx.x, rank, sl, g;
  if (b < R * Bp) {
    rank = b / Bp;
    sl = b % Bp;
    g = 0;
  } else {
    b -= R * Bp;
    const int per = Bp * (G - 1);
    rank = b / per;
    sl = (b % per) % Bp;
    g = 1 + (b % per) / Bp;
  }
  const LmRankArgs& a = A.r[rank];
  if (sl >= a.B) return;
  const int s = a.s0 + sl;
  StreamFrame& F = a.fr[s];
  if (!F.active) return;
  const size_t rb = (size_t)s * 2 * a.max_in;
  LmJob J;
  J.S = &F.lm[round];
  J.R = LmRecView{a.r_type + rb, a.r_px + rb, a.r_py + rb, a.r_pz + rb, a.r_a[0] + rb, a.r_a[1] + rb,
                  a.r_a[2] + rb, a.r_b[0] + rb, a.r_b[1] + rb, a.r_b[2] + rb};
  J.nrec = F.nc_stack + F.ns_stack;
  J.part = a.partials + (size_t)s * a.max_chunks * LM_NACC;
  J.sync = a.lm_sync + ((size_t)s * 2 + round) * LM_SYNC_WORDS;
  J.xpub = a.lm_xpub + ((size_t)s * 2 + round) * 8;
  J.best_out = F.pose;
  J.err = &F.err;
  J.err_code = MAP_ERR_LM_SYNC;
  J.prof = a.pdbg ? a.pdbg + 17 : nullptr;
  J.rank = rank;
  J.nrank = R;
  const size_t sr = (size_t)s * 2 + round;
  J.peer = A.peer + (((size_t)(F.epoch & 1u) * a.B * 2 + sr) * R) * LM_MAX_PASSES * LM_NACC;
  J.peer_flag = A.peer_flag + sr * R;
  J.flag_base = F.epoch * (uint32_t)LM_MAX_PASSES;
  lm_round_device<LM_THREADS>(J, g, G);
}

struct LmGroupCtx {
  int round, G;
  double* peer;
  uint32_t* peer_flag;
};
static void lm_group_launch(const void* const* blobs, int nrank, hipStream_t st, void* user) {
  const LmGroupCtx& C = *static_cast<const LmGroupCtx*>(user);
  LmGroupArgs A{};
  for (int r = 0; r < nrank; ++r) A.r[r] = *static_cast<const LmRankArgs*>(blobs[r]);
  A.peer = C.peer;
  A.peer_flag = C.peer_flag;
  A.nrank = nrank;
  k_lm_group<<<nrank * lm_padded(A.r[0].B) * C.G, LM_THREADS, 0, st>>>(A, C.round, C.G);
}

// sharded: every rank stores points with the same pose, so after the LM every rank adopts
// rank 0's (they are equal when the all-reduce is bit-identical on every rank, as RCCL's and
// the Python transports are); a rank that differed counts it in debug counter 40
__global__ void k_pose_publish(MapperDev D) {
  const int s = D.s0 + blockIdx.x, i = threadIdx.x;
  if (i < 7) D.pose_x[((size_t)D.rank * D.B + s) * 8 + i] = D.fr[s].pose[i];
}
__global__ void k_pose_adopt(MapperDev D) {
  const int s = D.s0 + blockIdx.x, i = threadIdx.x;
  StreamFrame& F = D.fr[s];
  if (i < 7) {
    const double v = D.pose_x[(size_t)s * 8 + i];  // rank 0's slot
    if (__double_as_longlong(v) != __double_as_longlong(F.pose[i])) atomicAdd(&D.dbg[40], 1ull);
    F.pose[i] = v;
  }
}

// which cube (if any) slot `slot` of (s, m) re-filters this frame; false: nothing to do.  A
// window cube that received nothing and whose content is a VoxelGrid fixed point keeps it:
// re-filtering it (laser_mapping.cpp:795-808) would reproduce it bit for bit.
__device__ inline bool revox_target(const MapperDev& D, int s, int m, int slot, int* cube_out, int* append_out) {
  const StreamFrame& F = D.fr[s];
  if (!F.active) return false;
  int cube, append;
  if (slot < F.valid_num) {
    cube = F.window[slot];
    append = 0;
  } else if (slot >= WIN_VALID_MAX && slot - WIN_VALID_MAX < min(F.extra_n[m], EXTRA_CAP)) {
    cube = F.extra_list[m][slot - WIN_VALID_MAX];
    append = 1;
  } else {
    return false;
  }
  const uint32_t* ioff = D.ins_off + sm_index(s, m) * (INS_SLOTS + 1);
  const uint32_t n_new = ioff[slot + 1] - ioff[slot];
  const uint2 cv = D.cube_tab[sm_index(s, m) * NCUBE + cube];
  if (!append && n_new == 0 && (cv.y == 0 || D.stable_tok[sm_index(s, m) * NCUBE + cube] == cv.x + 1))
    return false;
  *cube_out = cube;
  *append_out = append;
  return true;
}

// ---------------------------------------------------------------------------------------
// insertion of the stacks into the cube grid with the final pose (laser_mapping.cpp:741-788),
// then the inserted points grouped by target cube (stable counting sort); one workgroup per
// (stream, map): each re-VoxelGrid workgroup then reads one contiguous run, in input order
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(VX_THREADS) k_insert_bucket(MapperDev D) {
  __shared__ int cslot[NCUBE];
  __shared__ uint32_t base[INS_SLOTS];
  __shared__ uint32_t wcnt[VX_WAVES][INS_SLOTS];
  const int sm = 2 * D.s0 + blockIdx.x, s = sm >> 1, m = sm & 1;
  StreamFrame& F = D.fr[s];
  if (!F.active) return;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int n = m == 0 ? F.nc_stack : F.ns_stack;
  {
    // insertion of the stack into the cube grid with the final pose (laser_mapping.cpp:741-788):
    // the map-frame point and its cube; cubes outside the window that receive points are listed
    double X[7];
    for (int i = 0; i < 7; ++i) X[i] = F.pose[i];
    // transformUpdate (:147-151) for a frame queued behind this one (k_frame_prep); the host
    // computes the same at the end of the frame
    if (m == 0 && tid == 0) pose_transform_update(X, F.wodom, F.wmap);
    const int c0 = F.center[0], c1 = F.center[1], c2 = F.center[2];
    const int e0 = F.cen[0], e1 = F.cen[1], e2 = F.cen[2];
    const uint32_t epoch = F.epoch;
    // the stack points INS_LOADS at a time from a clamped index, all in flight before the first is
    // transformed (a load per loop trip is one memory latency per trip)
    constexpr int INS_LOADS = 4;
    const float4* stk = D.stack[m] + (size_t)s * D.max_in;
    for (int i0 = tid; i0 < n; i0 += INS_LOADS * VX_THREADS) {
      float4 q[INS_LOADS];
#pragma unroll
      for (int u = 0; u < INS_LOADS; ++u) q[u] = stk[min(i0 + u * VX_THREADS, n - 1)];
#pragma unroll
      for (int u = 0; u < INS_LOADS; ++u) {
        const int i = i0 + u * VX_THREADS;
        if (i >= n) break;
        const float4 sel = to_map(X, q[u]);
        const int ci = cube_of(sel.x, e0), cj = cube_of(sel.y, e1), ck = cube_of(sel.z, e2);
        int tag = -1;
        // sharded: only the owner of the point's 4 m block stores it (comm.h)
        const bool mine = !D.sharded || shard_owner(sel.x, sel.y, sel.z, 1.0f / D.leaf[m], D.blk_v[m], D.nrank) == D.rank;
        if (mine && ci >= 0 && ci < CW && cj >= 0 && cj < CH && ck >= 0 && ck < CD) {
          tag = ci + CW * cj + CW * CH * ck;
          const bool in_window = ci >= c0 - 2 && ci <= c0 + 2 && cj >= c1 - 2 && cj <= c1 + 2 && ck >= c2 - 1 && ck <= c2 + 1;
          if (!in_window) {
            uint32_t* fl = D.extra_flag + sm_index(s, m) * NCUBE + tag;
            if (atomicExch(fl, epoch) != epoch) {
              int e = atomicAdd(&F.extra_n[m], 1);
              if (e < EXTRA_CAP) F.extra_list[m][e] = tag;
              else atomicOr(&F.err, MAP_ERR_EXTRA);
            }
          }
        }
        const size_t o = sm_index(s, m) * D.max_in + i;
        D.ins_pts[o] = sel;
        D.ins_tag[o] = tag;
      }
    }
    __syncthreads();  // the points, tags and the out-of-window list, for the grouping below
  }
  // group the inserted points by target cube (stable counting sort): each re-VoxelGrid
  // workgroup then reads one contiguous run, in input order
  const int* tag = D.ins_tag + sm_index(s, m) * D.max_in;
  const float4* pts = D.ins_pts + sm_index(s, m) * D.max_in;
  float4* out = D.ins_sorted + sm_index(s, m) * D.max_in;
  uint32_t* off = D.ins_off + sm_index(s, m) * (INS_SLOTS + 1);
  for (int c = tid; c < NCUBE; c += VX_THREADS) cslot[c] = -1;
  for (int k = tid; k < INS_SLOTS; k += VX_THREADS) base[k] = 0;
  __syncthreads();
  const int vn = F.valid_num, ne = min(F.extra_n[m], EXTRA_CAP);
  if (tid < vn) cslot[F.window[tid]] = tid;
  if (tid < ne) cslot[F.extra_list[m][tid]] = WIN_VALID_MAX + tid;
  // this thread's slot (tid < INS_SLOTS) for the re-VoxelGrid list below: its cube's table entry and
  // token are loaded now, their latency hidden behind the grouping (the revox_target test)
  int my_cube = -1;
  if (tid < vn) my_cube = F.window[tid];
  else if (tid >= WIN_VALID_MAX && tid < WIN_VALID_MAX + ne) my_cube = F.extra_list[m][tid - WIN_VALID_MAX];
  uint2 my_cv = make_uint2(0u, 0u);
  uint32_t my_tok = 0u;
  if (my_cube >= 0) {
    my_cv = D.cube_tab[sm_index(s, m) * NCUBE + my_cube];
    my_tok = D.stable_tok[sm_index(s, m) * NCUBE + my_cube];
  }
  __syncthreads();
  for (int i = tid; i < n; i += VX_THREADS) {
    const int t = tag[i];
    const int sl = t >= 0 ? cslot[t] : -1;
    if (sl >= 0) atomicAdd(&base[sl], 1u);
  }
  __syncthreads();
  const uint32_t my_new = tid < INS_SLOTS ? base[tid] : 0u;  // points inserted into this slot's cube
  __syncthreads();  // (every count read before the scan below rewrites base)
  if (wid == 0) {  // exclusive scan of the slot counts by one wave: lane l owns slots l*PL ..
    constexpr int PL = (INS_SLOTS + 63) / 64;
    uint32_t c[PL], sum = 0;
#pragma unroll
    for (int u = 0; u < PL; ++u) {
      const int k = lane * PL + u;
      c[u] = k < INS_SLOTS ? base[k] : 0u;
      sum += c[u];
    }
    uint32_t x = sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    uint32_t acc = x - sum;
#pragma unroll
    for (int u = 0; u < PL; ++u) {
      const int k = lane * PL + u;
      if (k < INS_SLOTS) {
        base[k] = acc;
        off[k] = acc;
      }
      acc += c[u];
    }
    if (lane == 63) off[INS_SLOTS] = x;
  }
  __syncthreads();
  // software pipeline: the next chunk's tag and point are loaded while this chunk is grouped
  int t_next = tid < n ? tag[tid] : -1;
  float4 p_next = tid < n ? pts[tid] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int c0 = 0; c0 < n; c0 += VX_THREADS) {
    const int i = c0 + tid;
    const int t = t_next;
    const float4 p_cur = p_next;
    t_next = -1;  // (past the end: no point)
    if (i + VX_THREADS < n) {
      t_next = tag[i + VX_THREADS];
      p_next = pts[i + VX_THREADS];
    }
    const int sl = t >= 0 ? cslot[t] : -1;
    for (int k = tid; k < VX_WAVES * INS_SLOTS; k += VX_THREADS) (&wcnt[0][0])[k] = 0;
    __syncthreads();
    // rank among the lanes of this wave with the same slot (peel one slot value per pass)
    uint32_t rank = 0;
    bool pending = sl >= 0;
    while (true) {
      const uint64_t live = __ballot(pending);
      if (!live) break;
      const int leader = __ffsll((unsigned long long)live) - 1;
      const int lsl = __shfl(sl, leader, 64);
      const bool mine = pending && sl == lsl;
      const uint64_t mk = __ballot(mine);
      if (mine) {
        rank = __popcll(mk & lanemask_lt());
        pending = false;
      }
      if (lane == 0) wcnt[wid][lsl] = __popcll(mk);
    }
    __syncthreads();
    if (tid < INS_SLOTS) {  // wave prefix per slot, advance the slot base
      uint32_t acc = base[tid];
      for (int w = 0; w < VX_WAVES; ++w) {
        const uint32_t c = wcnt[w][tid];
        wcnt[w][tid] = acc;
        acc += c;
      }
      base[tid] = acc;
    }
    __syncthreads();
    if (sl >= 0) out[wcnt[wid][sl] + rank] = p_cur;
    __syncthreads();
  }
  // this (stream, map)'s re-VoxelGrid items, listed by size class (k_revox takes the largest
  // first); the test is revox_target's: a window cube that received nothing and holds fixed-point
  // (or no) content is skipped
  static_assert(INS_SLOTS <= VX_THREADS, "one thread per slot");
  if (my_cube >= 0) {
    const bool append = tid >= WIN_VALID_MAX;
    if (append || my_new != 0 || (my_cv.y != 0 && my_tok != my_cv.x + 1)) {
      const uint32_t nt = my_cv.y + my_new;
      const int c = nt < 1024u ? 0 : min(RQ_CLASSES - 1, 32 - __clz(nt >> 10));
      const uint32_t k = atomicAdd(&D.rq_ctl[c], 1u);
      D.rq[(size_t)c * D.rq_cap + k] = (uint32_t)(sm * INS_SLOTS + tid);
    }
  }
}

// ---------------------------------------------------------------------------------------
// re-VoxelGrid of every window cube (old content ++ inserted points, :795-808); cubes outside
// the window that received points get them appended raw (:762).  One workgroup per cube:
// the merge path (a fixed-point cube plus a few new points, voxel.h vx_merge_fixed_point) or
// the full filter in a VX_THREADS workgroup with the whole LDS, then the cube's cell index.
// ---------------------------------------------------------------------------------------
#ifndef REVOX_PROF_MIN_N
#define REVOX_PROF_MIN_N 0  // diagnostics builds: phase counters of the items of at least this many points only
#endif
template <bool PCL>
__device__ inline void revox_item(MapperDev& D, int s, int m, int slot, int cube, int append, uint32_t* lds) {
  constexpr int LW = VX_LDS_WORDS;
  StreamFrame& F = D.fr[s];
  const uint32_t* ioff = D.ins_off + sm_index(s, m) * (INS_SLOTS + 1);
  const uint32_t i0 = ioff[slot], n_new = ioff[slot + 1] - i0;
  uint32_t* tok = D.stable_tok + sm_index(s, m) * NCUBE + cube;
  uint2* tab = D.cube_tab + sm_index(s, m) * NCUBE;
  const uint2 cv = tab[cube];
  if (cv.y + n_new < (uint32_t)REVOX_PROF_MIN_N) D.pdbg = nullptr;
  float4* ar = arena_base(D, s, m, F.arena_active[m]);
  VoxSeg S;
  S.src0 = ar + cv.x;
  S.n0 = (int)cv.y;
  S.src1 = D.ins_sorted + sm_index(s, m) * D.max_in + i0;
  S.tag1 = nullptr;
  S.n1 = (int)n_new;
  S.tag = cube;
  S.leaf = D.leaf[m];
  S.append_only = append;
  S.out = ar;
  S.tail = &F.arena_tail[m];
  S.cap = D.map_cap;
  S.res_off = &tab[cube].x;
  S.res_cnt = &tab[cube].y;
  S.stable_out = tok;
  S.scratch_pts = D.vx_pts + sm_index(s, m) * D.scratch_cap;
  S.scratch_idx = D.vx_idx + sm_index(s, m) * D.scratch_cap;
  S.scratch_tail = &F.scratch_tail[m];
  S.scratch_cap = D.scratch_cap;
  S.err = &F.err;
  S.prof = D.pdbg ? D.pdbg + 11 : nullptr;  // merge phases: dbg[11..14]
  S.anchored = 1;  // a merge keys the voxels from the cube's corner (VoxSeg::anchored)
  cube_corner(cube, F.cen, S.anchor);
  bool merged = false;
  const unsigned long long t0 = __builtin_readcyclecounter();
  const bool fixed = n_new > 0 && n_new <= VX_MERGE_CAP && cv.y > 0 && *tok == cv.x + 1;
  if (PCL && !append) {
    // PCL's summation order (exact_voxel_order): also a window cube that received nothing but
    // is not a VoxelGrid fixed point (raw appended content, content set through the API), as the
    // reference re-filters every window cube (:795-808)
    uint32_t* sb = lds + LW - 3;
    const uint32_t n = cv.y + n_new;
    if (threadIdx.x == 0) *sb = atomicAdd(&F.hot_tail[m], n + MP_SLACK);
    __syncthreads();
    const uint32_t so = *sb;
    __syncthreads();
    bool global = n > (uint32_t)VH_BIG_N;
    uint32_t reuse_off = 0xFFFFFFFFu, reuse_cnt = 0;
    if (!global) {
      // the input-order filter sums every voxel of at most 2 members (order-free) and records the
      // others, then voxel_hot.h sums those in std::sort's order
      if ((size_t)so + n + MP_SLACK > mp_cube_scratch(D)) {
        if (threadIdx.x == 0) atomicOr(&F.err, MAP_ERR_SORT);
      } else {
        S.hot = map_hot(D, sm_index(s, m), so, n);
        if (fixed) {
          merged = vx_merge_fixed_point<VX_THREADS, (int)VX_MERGE_CAP, VX_LDS_WORDS, true>(S, lds);
          __syncthreads();  // false: grid overflow, full filter below
        }
        if (!merged) voxel_segment(S, lds);
        const VxSrc P{ar + cv.x, (int)cv.y, D.ins_sorted + sm_index(s, m) * D.max_in + i0};
        const int he = vh_fixup<VX_THREADS>(P, (int)n, ar, S.hot, lds, LW - 256, *reinterpret_cast<VxMisc*>(lds + LW - 192),
                                            tok, &F.err, D.pdbg ? D.pdbg + 50 : nullptr,
                                            D.pdbg ? D.pdbg + 72 : nullptr, D.pdbg ? D.pdbg + 82 : nullptr);
        // (over VH_MAX_N, a part too large for the LDS after the first partition: the global
        // sort below writes the cube again, into the block the filter above allocated for it:
        // the same voxels, so the same count)
        global = he < 0;
        __syncthreads();
        if (global) {
          const uint2 v = tab[cube];  // (thread 0 wrote it inside the filter, before the barrier)
          reuse_off = v.x;
          reuse_cnt = v.y;
        }
      }
    }
    if (global) {  // the whole std::sort emulated in global memory (voxel_pcl.h)
      VxPclOut O;
      O.reuse_off = reuse_off;
      O.reuse_cnt = reuse_cnt;
      O.out = ar;
      O.tail = &F.arena_tail[m];
      O.cap = D.map_cap;
      O.res_off = &tab[cube].x;
      O.res_cnt = &tab[cube].y;
      O.stable_out = tok;
      map_voxel_pcl(D, sm_index(s, m), so, VxSrc{ar + cv.x, (int)cv.y, D.ins_sorted + sm_index(s, m) * D.max_in + i0},
                    (int)n, D.leaf[m], O, lds, &F.err);
    }
    __syncthreads();
  } else {
    if (!append && fixed) {
      merged = vx_merge_fixed_point(S, lds);
      __syncthreads();  // false: grid overflow, full filter below
    }
    if (!merged) voxel_segment(S, lds);
    __syncthreads();
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  // the cube's new content -> its cell index (cubeindex.h)
  uint32_t* res = lds + LW - 2;
  if (threadIdx.x == 0) {
    const uint2 v = tab[cube];  // written by this thread inside the filter
    res[0] = v.x;
    res[1] = v.y;
  }
  __syncthreads();
  const uint32_t off = res[0], n = res[1];
  __syncthreads();  // res may lie in the index build's LDS
  int corner[3];
  cube_corner(cube, F.cen, corner);
  if (!cube_index_build<VX_THREADS, CI_LDS_MAX_T>(ar + off, n, corner, carena_base(D, s, m, F.arena_active[m]) + off,
                                  ctab_base(D, s, m, F.arena_active[m]) + 4 * (size_t)off, lds, D.pdbg ? D.pdbg + 16 : nullptr) &&
      threadIdx.x == 0)
    atomicOr(&F.err, MAP_ERR_INDEX);
  // read old content + new points, write the filtered cube, then its index (read it, write
  // the cell-sorted copy and the table)
  if (threadIdx.x == 0)
    atomicAdd(&F.vx_bytes, 16ull * (cv.y + n_new) + 16ull * 3 * n + (n ? 8ull * ci_table_size(n) : 0ull));
  if (threadIdx.x == 0 && D.pdbg) {
    const unsigned long long t2 = __builtin_readcyclecounter();
    const int k = merged ? 0 : (append ? 2 : 1);
    atomicAdd(&D.dbg[k], t1 - t0);       // filter cycles: merge / full / append
    atomicAdd(&D.dbg[4 + k], 1ull);      // items
    atomicAdd(&D.dbg[8], t2 - t1);       // index build cycles
    atomicAdd(&D.dbg[9], (unsigned long long)n);
    atomicAdd(&D.dbg[10], (unsigned long long)cv.y);
    int hb = 0;
    while (hb < 7 && n >= (1024u << hb)) ++hb;
    atomicAdd(&D.dbg[24 + hb], 1ull);
    atomicAdd(&D.dbg[32 + hb], t2 - t0);
    if (merged) {
      atomicAdd(&D.dbg[3], (unsigned long long)n_new);  // new points of merged cubes
      atomicAdd(&D.dbg[7], 1ull);                       // merges
    }
  }
}

// One workgroup per item (no loop over items: a loop around revox_item spills hundreds of
// registers): workgroup b takes the b-th item of the frame's list (k_insert_bucket), largest size
// class first, so the longest items are dispatched first; workgroups past the list's end leave
// after one load.  PCL: exact_voxel_order (its own instantiation, so that the sort's registers do
// not weigh on the input-order kernel)
template <bool PCL>
__global__ void __launch_bounds__(VX_THREADS) k_revox(MapperDev D) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[VX_LDS_WORDS];
  uint32_t b = blockIdx.x;
  int item = -1;
  for (int c = RQ_CLASSES - 1; c >= 0; --c) {
    const uint32_t nc = D.rq_ctl[c];
    if (b < nc) {
      item = (int)D.rq[(size_t)c * D.rq_cap + b];
      break;
    }
    b -= nc;
  }
  if (item < 0) return;
  const int slot = item % INS_SLOTS, sm = item / INS_SLOTS;
  int cube = 0, append = 0;
  if (!revox_target(D, sm >> 1, sm & 1, slot, &cube, &append)) return;
  revox_item<PCL>(D, sm >> 1, sm & 1, slot, cube, append, lds);
}

// cell index of one cube whose content was set through the API (cen: the host's grid centre)
__global__ void __launch_bounds__(VX_THREADS) k_cube_index(MapperDev D, int s, int m, int c0, int c1,
                                                           int3 cen) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[CI_LDS_MAX_T + VX_WAVES + 1];
  const int cube = c0 + blockIdx.x;
  if (cube >= c1) return;
  StreamFrame& F = D.fr[s];
  const uint2 cv = D.cube_tab[sm_index(s, m) * NCUBE + cube];
  if (cv.y == 0) return;
  const int cenv[3] = {cen.x, cen.y, cen.z};
  int corner[3];
  cube_corner(cube, cenv, corner);
  const int active = F.arena_active[m];
  if (!cube_index_build<VX_THREADS>(arena_base(D, s, m, active) + cv.x, cv.y, corner,
                                    carena_base(D, s, m, active) + cv.x,
                                    ctab_base(D, s, m, active) + 4 * (size_t)cv.x, lds) &&
      threadIdx.x == 0)
    atomicOr(&F.err, MAP_ERR_INDEX);
}

// ---------------------------------------------------------------------------------------
// arena compaction: live cubes copied, in cube order, into the other arena
// ---------------------------------------------------------------------------------------
// Launched over every (stream, map) pair sm = 2 s0 + b of the handle; a pair whose tail is at
// or below compact_at exits at once (the decision is taken on the device, from the records)
__device__ inline bool compact_due(const MapperDev& D, int sm) {
  return D.fr[sm >> 1].arena_tail[sm & 1] > D.compact_due_at;
}

__global__ void k_compact_scan(MapperDev D, uint32_t* new_off) {
  // one workgroup (1024 threads) per pair
  __shared__ uint32_t ws[VX_WAVES + 1];
  const int sm = 2 * D.s0 + blockIdx.x;
  if (!compact_due(D, sm)) return;
  const uint2* tab = D.cube_tab + (size_t)sm * NCUBE;
  uint32_t* no = new_off + (size_t)blockIdx.x * (NCUBE + 1);
  constexpr int PER = (NCUBE + VX_THREADS - 1) / VX_THREADS;  // 5
  uint32_t v[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    int c = threadIdx.x * PER + k;
    v[k] = c < NCUBE ? tab[c].y : 0u;
    sum += v[k];
  }
  uint32_t total;
  uint32_t pre = vx_block_scan(sum, ws, &total);
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    int c = threadIdx.x * PER + k;
    if (c < NCUBE) no[c] = pre;
    pre += v[k];
  }
  if (threadIdx.x == 0) no[NCUBE] = total;
}

__global__ void k_compact_copy(MapperDev D, const uint32_t* new_off) {
  const int p = blockIdx.y, sm = 2 * D.s0 + p;
  if (!compact_due(D, sm)) return;
  const int s = sm >> 1, m = sm & 1;
  StreamFrame& F = D.fr[s];
  uint2* tab = D.cube_tab + (size_t)sm * NCUBE;
  const uint32_t* no = new_off + (size_t)p * (NCUBE + 1);
  const float4* src = arena_base(D, s, m, F.arena_active[m]);
  float4* dst = arena_base(D, s, m, 1 - F.arena_active[m]);
  const float4* csrc = carena_base(D, s, m, F.arena_active[m]);
  float4* cdst = carena_base(D, s, m, 1 - F.arena_active[m]);
  const uint2* tsrc = ctab_base(D, s, m, F.arena_active[m]);
  uint2* tdst = ctab_base(D, s, m, 1 - F.arena_active[m]);
  for (int c = blockIdx.x; c < NCUBE; c += gridDim.x) {
    const uint2 cv = tab[c];
    for (uint32_t i = threadIdx.x; i < cv.y; i += blockDim.x) {
      dst[no[c] + i] = src[cv.x + i];
      cdst[no[c] + i] = csrc[cv.x + i];  // the cell index moves verbatim (offsets are local)
    }
    if (cv.y) {
      const uint32_t T = ci_table_size(cv.y);
      for (uint32_t h = threadIdx.x; h < T; h += blockDim.x) tdst[4 * (size_t)no[c] + h] = tsrc[4 * (size_t)cv.x + h];
    }
  }
}

__global__ void k_compact_commit(MapperDev D, const uint32_t* new_off) {
  __shared__ int due;
  const int p = blockIdx.x, sm = 2 * D.s0 + p;
  if (threadIdx.x == 0) due = compact_due(D, sm);
  __syncthreads();  // thread 0 moves the tail below
  if (!due) return;
  const int s = sm >> 1, m = sm & 1;
  StreamFrame& F = D.fr[s];
  uint2* tab = D.cube_tab + (size_t)sm * NCUBE;
  const uint32_t* no = new_off + (size_t)p * (NCUBE + 1);
  uint32_t* tok = D.stable_tok + (size_t)sm * NCUBE;
  for (int c = threadIdx.x; c < NCUBE; c += blockDim.x) {
    const bool stable = tok[c] != 0 && tok[c] == tab[c].x + 1;  // content moves verbatim
    tab[c].x = no[c];
    tok[c] = stable ? no[c] + 1 : 0u;
  }
  if (threadIdx.x == 0) {
    F.arena_tail[m] = no[NCUBE];
    F.arena_active[m] = 1 - F.arena_active[m];
    if (no[NCUBE] > D.compact_at) atomicOr(&F.err, MAP_ERR_LIVE);  // the live map itself
    atomicAdd(&D.dbg[41], 1ull);
    atomicAdd(&D.dbg[48 + m], 1ull);  // per map
  }
}

// ---------------------------------------------------------------------------------------
// publish-side outputs (laser_mapping.cpp:884-911)
// ---------------------------------------------------------------------------------------
// laserCloudMap = corner cube 0, surf cube 0, corner cube 1, ... (:886-891): offsets of every
// (cube, map) run, one workgroup
__global__ void __launch_bounds__(VX_THREADS) k_map_scan(MapperDev D, int s, uint32_t* off) {
  __shared__ uint32_t ws[VX_WAVES + 1];
  const uint2* tc = D.cube_tab + sm_index(s, 0) * NCUBE;
  const uint2* ts = D.cube_tab + sm_index(s, 1) * NCUBE;
  constexpr int PER = (NCUBE + VX_THREADS - 1) / VX_THREADS;
  uint32_t v[2 * PER], sum = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int c = threadIdx.x * PER + k;
    v[2 * k] = c < NCUBE ? tc[c].y : 0u;
    v[2 * k + 1] = c < NCUBE ? ts[c].y : 0u;
    sum += v[2 * k] + v[2 * k + 1];
  }
  uint32_t total;
  uint32_t pre = vx_block_scan(sum, ws, &total);
#pragma unroll
  for (int k = 0; k < 2 * PER; ++k) {
    const int c = threadIdx.x * PER + k / 2;
    if (c < NCUBE) off[2 * c + (k & 1)] = pre;
    pre += v[k];
  }
  if (threadIdx.x == 0) off[2 * NCUBE] = total;
}

__global__ void k_map_gather(MapperDev D, int s, const uint32_t* off, float4* out) {
  const StreamFrame& F = D.fr[s];
  for (int e = blockIdx.x; e < 2 * NCUBE; e += gridDim.x) {
    const int c = e >> 1, m = e & 1;
    const uint2 cv = D.cube_tab[sm_index(s, m) * NCUBE + c];
    const float4* src = arena_base(D, s, m, F.arena_active[m]) + cv.x;
    for (uint32_t i = threadIdx.x; i < cv.y; i += blockDim.x) out[off[e] + i] = src[i];
  }
}

// laserCloudFullRes registered with the mapped pose: pointAssociateToMap (:154-164, :901-905)
__global__ void k_register(const float4* in, float4* out, int n, MapPose P) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = to_map(P.x, in[i]);
}

// ---------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------
// page-locked host array (hipHostMalloc) with the few vector operations used here
template <typename T>
struct PinnedArray {
  T* p = nullptr;
  size_t n = 0;
  ~PinnedArray() { release(); }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    n = 0;
  }
  bool assign(size_t count, const T& v, unsigned flags = hipHostMallocDefault) {
    release();
    if (hipHostMalloc(reinterpret_cast<void**>(&p), sizeof(T) * std::max<size_t>(count, 1), flags) != hipSuccess) {
      p = nullptr;
      return false;
    }
    n = count;
    for (size_t i = 0; i < n; ++i) p[i] = v;
    return true;
  }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
  T* data() { return p; }
  size_t size() const { return n; }
};

struct HostStream {
  double q_wmap_wodom[4] = {0, 0, 0, 1}, t_wmap_wodom[3] = {0, 0, 0};
  double q_wodom[4] = {0, 0, 0, 1}, t_wodom[3] = {0, 0, 0};
  double pose[7] = {0, 0, 0, 1, 0, 0, 0};
  double q_hf[4] = {0, 0, 0, 1}, t_hf[3] = {0, 0, 0};
  bool pending = false, skip = false;
  bool solved_last = false;  // solved by the last loam_mapper_solve (loam_mapper_total_iterations)
  // the input of the next solve (LaserMapping::input, laser_mapping.cpp:178-209), kept apart from
  // the frame in flight (loam_mapper_solve_async) until that solve takes it
  bool in_ready = false;
  bool stk_launched = false;  // its stack VoxelGrid already queued (loam_mapper_prefetch)
  unsigned long long stk_seq = 0;  // that stack launch (k_stack_done)
  const float4* in_p[2] = {nullptr, nullptr};
  int in_n[2] = {0, 0};
  double in_q[4] = {0, 0, 0, 1}, in_t[3] = {0, 0, 0};
  int frame = 0;
  int cen[3] = {10, 10, 5};  // laserCloudCen* after the stream's last finished frame
  loam_map_stats st{};
};

// device error flags of a stream -> message (VX_ERR_* of voxel.h, MAP_ERR_* above)
inline std::string map_err_text(int e) {
  std::string m;
  auto add = [&](int bit, const char* what) {
    if (e & bit) m += (m.empty() ? "" : ", ") + std::string(what);
  };
  add(VX_ERR_CAPACITY, "VoxelGrid scratch full");
  add(VX_ERR_OUTPUT, "map arena full (max_map_points)");
  add(MAP_ERR_SUBMAP, "submap larger than max_submap_points");
  add(MAP_ERR_EXTRA, "too many out-of-window insertions");
  add(MAP_ERR_HASH, "cell table full");
  add(MAP_ERR_LM_SYNC, "LM workgroup hand-off timed out");
  add(MAP_ERR_INDEX, "cube cell index capacity");
  add(MAP_ERR_LIVE, "live map larger than the arena's compaction bound");
  add(MAP_ERR_SORT, "PCL-order VoxelGrid input larger than its sort lists / scratch");
  add(MAP_ERR_STACK, "split stack VoxelGrid: a range has more voxels than its LDS groups");
  add(MAP_ERR_STACK_WAIT, "the frame's stack VoxelGrid did not finish in time (device wait)");
  add(VH_ERR_ROOTS | VH_ERR_LIST, "PCL-order VoxelGrid sort lists full");
  add(VH_ERR_SPIN, "PCL-order VoxelGrid sort: a wave's wait for a listed subtree ran out");
  return m + " (flags " + std::to_string(e) + ")";
}

}  // namespace loam

using namespace loam;

enum : int { FAM_STACK = 0, FAM_HASH, FAM_CORR, FAM_LM, FAM_INSERT, FAM_REVOX, FAM_OTHER, NFAM };

// a frame in flight (loam_mapper_solve_async): what its streams were given, where its records
// come back (the D2H buffer of its stack parity), and whether it was queued behind another
// frame with its records prepared on the device (chained)
struct FrameRec {
  bool chained = false, graph = false;
  bool has_deferred = false;  // known (its records are back) to have deferred streams
  bool pending = false;       // not enqueued yet: inputs and stack taken, run on the host path later
  bool behind = false;        // solve_async was called with another frame in the queue
  bool early_seen = false;    // its poses and stats were taken from the early records (loam_mapper_solve_pose)
  uint32_t epoch = 0;         // its frame number (the done word frame_out writes)
  int fpar = 0;
  uint64_t seq = 0;  // enqueue order (0: nothing was enqueued)
  std::vector<int> active;
  std::vector<std::array<double, 7>> wodom;
  std::vector<std::array<const float4*, 2>> in_p;
  std::vector<std::array<int, 2>> in_n;
  std::vector<unsigned long long> stk_seq;
};

struct loam_mapper {
  // the status of a frame loam_mapper_solve_async finished to make room (LOAM_ERR_CAPACITY /
  // _SYNC), held for the next loam_mapper_wait / loam_mapper_solve (as LOAM_ERR_EARLIER): the
  // solve_async that finished it returns OK, since it did enqueue its own frame
  int32_t held_rc = 0;
  std::string held_msg;
  loam_params P;
  bool prof = false;
  std::vector<hipEvent_t> ev_pool;
  std::vector<int> ev_fam;  // family of each recorded (start, stop) pair
  double fam_ms[NFAM] = {0}, fam_bytes[NFAM] = {0};
  long long fam_launches[NFAM] = {0};
  int dev = 0, B = 1;
  hipStream_t st = nullptr;
  hipStream_t st2 = nullptr;  // stack VoxelGrid, concurrent with the submap / hash build
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  MapperDev D{};
  PinnedArray<StreamFrame> hf;  // pinned: the per-frame H2D / D2H of the stream records
  std::vector<HostStream> hs;
  uint2* cube_tab[2] = {nullptr, nullptr};
  int parity = 0;
  uint32_t* tok_tmp = nullptr;  // [B][2][NCUBE] the shifted fixed-point tokens
  uint32_t* d_new_off = nullptr;
  std::vector<void*> allocs;
  uint32_t frame_counter = 0;
  int n_cu = 256;  // compute units (grid of the worklist kernels)
  // compact an arena once its tail passes this: one frame writes at most the window content
  // (<= max_submap_points) plus the stack (<= max_input_points) plus the few cubes outside
  // the window that receive points; a write past the capacity is reported (err flags)
  uint32_t compact_at = 0;
  int lm_G = 0;  // workgroups per stream of k_lm_round (0: two-kernel path k_lm_eval / k_lm_step)
  bool want_ipc = false;            // cross-process ranks: set up the IPC peer buffers at create
  void* ipc_own = nullptr;          // this rank's LM peer buffer (ipc_peer_setup)
  std::vector<void*> ipc_open;      // the other ranks' buffers, mapped from their IPC handles
  int knn_cs = 0;     // k_knn: 8 lanes per query splitting the cells (handles of <= 4 streams), else 0
                      // (one lane per query)
  loam_comm* comm = nullptr;  // sharded mode (loam_mapper_create_sharded)
  PinnedArray<int> q_off;     // [B + 1] query offsets of the sharded kNN exchange
  int* d_q_off = nullptr;
  // hipGraph of the whole per-frame sequence (handles of <= 4 streams): one per cube-table
  // parity, used for frames without recentering, compaction, profiling or sharding
  int use_graph = 0;
  hipGraphExec_t gexec[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};  // [cube parity][stack parity]
  // stack VoxelGrids ahead of their frame (loam_mapper_prefetch / loam_mapper_solve_async):
  // stacks, their inputs and counts double-buffered by stack parity; spar: the next frame's
  int spar = 0, last_spar = 0;
  // frames in flight, oldest first: at most two, the second queued behind the first on the
  // device (loam_mapper_solve_async on a graph-path handle, its records from k_frame_prep)
  std::deque<FrameRec> q;
  uint64_t seq = 0, mirror_seq = 0;  // hf mirrors the device records as of frame mirror_seq
  PinnedArray<StreamFrame> hfo[2];   // [stack parity] the records after that parity's frame
  PinnedArray<FrameIn> fin[2];       // [stack parity] the graph path's frame inputs (k_frame_prep)
  const FrameIn* fin_dev[2] = {nullptr, nullptr};
  hipEvent_t ev_fr[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};  // [parity] frame start / records back (timed)
  unsigned long long stack_seq = 0;
  unsigned long long* d_stk_ready = nullptr;  // [2 parities]
  PinnedArray<unsigned long long> done;  // [2 parities]
  unsigned long long* done_dev = nullptr;
  StreamFrame* hfo_dev[2] = {nullptr, nullptr};
  // loam_mapper_solve_pose: graph-path frames also write their records after the second LM round
  // (before the insertion and re-VoxelGrid) with their own done word
  bool early = false;
  PinnedArray<StreamFrame> hfo_early[2];
  PinnedArray<unsigned long long> done_early;
  StreamFrame* hfo_early_dev[2] = {nullptr, nullptr};
  unsigned long long* done_early_dev = nullptr;
  uint32_t grow_max = 0;     // largest arena growth of one frame seen (compaction foresight)
  std::vector<std::array<uint32_t, 2>> last_tail;
  hipEvent_t ev_stack = nullptr;   // after the last stack launch (on st2)
  hipEvent_t ev_sin[2] = {nullptr, nullptr};  // the H2D of hsin[parity] done
  float4* stack_buf[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};  // [parity][map]
  int* stk_n_buf[2] = {nullptr, nullptr};
  int* stk_err_buf[2] = {nullptr, nullptr};
  StackIn* sin_buf[2] = {nullptr, nullptr};
  PinnedArray<StackIn> hsin[2];
  // publish-side buffers (grown on demand)
  uint32_t* d_map_off = nullptr;  // [2 * NCUBE + 1]
  float4* d_pub = nullptr;
  size_t pub_cap = 0;
};

namespace {

template <typename T>
int32_t dalloc(loam_mapper* h, T** p, size_t count) {
  void* q = nullptr;
  size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
  LOAM_HIP(hipMalloc(&q, bytes));
  // zero on the handle's own (non-blocking) stream: a null-stream memset is not ordered
  // before this stream's kernels; create() synchronizes the stream before returning
  LOAM_HIP(hipMemsetAsync(q, 0, bytes, h->st));
  h->allocs.push_back(q);
  *p = reinterpret_cast<T*>(q);
  return LOAM_OK;
}

uint32_t next_pow2(uint32_t v) {
  uint32_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

void free_all(loam_mapper* h) {
  if (h->D.lm_peer && h->comm) {  // the group's LM peer buffer (kernels done: the caller synchronized)
    comm_peer_release(h->comm);
    h->D.lm_peer = nullptr;
    h->D.lm_peer_flag = nullptr;
  }
  for (void* p : h->ipc_open) (void)hipIpcCloseMemHandle(p);
  h->ipc_open.clear();
  if (h->ipc_own) (void)hipFree(h->ipc_own);
  h->ipc_own = nullptr;
  h->D.ipc_tab = nullptr;
  for (void* p : h->allocs) (void)hipFree(p);
  h->allocs.clear();
  if (h->d_pub) (void)hipFree(h->d_pub);
  h->d_pub = nullptr;
  h->pub_cap = 0;
  for (auto& gp : h->gexec)
    for (auto& g : gp)
      if (g) (void)hipGraphExecDestroy(g);
  for (auto& e : h->ev_pool) (void)hipEventDestroy(e);
  if (h->ev_stack) (void)hipEventDestroy(h->ev_stack);
  for (auto& e : h->ev_sin)
    if (e) (void)hipEventDestroy(e);
  for (auto& ep : h->ev_fr)
    for (auto& e : ep)
      if (e) (void)hipEventDestroy(e);
  h->ev_pool.clear();
  for (auto& e : h->ev)
    if (e) (void)hipEventDestroy(e);
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->st) (void)hipStreamDestroy(h->st);
  if (h->st2) (void)hipStreamDestroy(h->st2);
}

void host_initial_guess(HostStream& H, double* pose) {
  // LaserMapping::input (laser_mapping.cpp:206-207)
  dq qm{H.q_wmap_wodom[0], H.q_wmap_wodom[1], H.q_wmap_wodom[2], H.q_wmap_wodom[3]};
  dq qo{H.q_wodom[0], H.q_wodom[1], H.q_wodom[2], H.q_wodom[3]};
  dq q = qmul(qm, qo);
  d3 r = qrot(qm, d3{H.t_wodom[0], H.t_wodom[1], H.t_wodom[2]});
  pose[0] = q.x; pose[1] = q.y; pose[2] = q.z; pose[3] = q.w;
  pose[4] = r.x + H.t_wmap_wodom[0];
  pose[5] = r.y + H.t_wmap_wodom[1];
  pose[6] = r.z + H.t_wmap_wodom[2];
}

void host_transform_update(HostStream& H) {
  // LaserMapping::transformUpdate (laser_mapping.cpp:147-151)
  dq qw{H.pose[0], H.pose[1], H.pose[2], H.pose[3]};
  dq qo{H.q_wodom[0], H.q_wodom[1], H.q_wodom[2], H.q_wodom[3]};
  dq qm = qmul(qw, qinv(qo));
  d3 r = qrot(qm, d3{H.t_wodom[0], H.t_wodom[1], H.t_wodom[2]});
  H.q_wmap_wodom[0] = qm.x; H.q_wmap_wodom[1] = qm.y; H.q_wmap_wodom[2] = qm.z; H.q_wmap_wodom[3] = qm.w;
  H.t_wmap_wodom[0] = H.pose[4] - r.x;
  H.t_wmap_wodom[1] = H.pose[5] - r.y;
  H.t_wmap_wodom[2] = H.pose[6] - r.z;
}

int32_t check_stream(loam_mapper* h, int32_t s) {
  if (!h) {
    set_error("null mapper handle");
    return LOAM_ERR_ARG;
  }
  if (s < 0 || s >= h->B) {
    set_error("stream index out of range");
    return LOAM_ERR_ARG;
  }
  return LOAM_OK;
}

}  // namespace

extern "C" {

// The persistent LM across processes (the peer one-shot reduce instead of an RCCL
// all-reduce per LM iteration): every rank allocates its LM peer buffer, exports it as an IPC handle,
// the handles travel through the comm's own all-gather, and every rank maps the others'.  All ranks
// take the same decision (each one's outcome is all-gathered): on any failure every rank keeps the
// two-kernel path.  Returns LOAM_OK with D.ipc_tab set, or LOAM_OK without it (fall back), or the
// comm's error.
static int32_t ipc_peer_setup(loam_mapper* h) {
  loam_comm* c = h->comm;
  MapperDev& D = h->D;
  const int R = c->size, me = c->rank;
  const size_t B = h->B, nslot = 2 * B * 2 * LM_MAX_PASSES * LM_NACC;
  const size_t bytes = nslot * sizeof(double) + B * 2 * sizeof(uint32_t);
  struct Msg {
    hipIpcMemHandle_t hdl;
    int32_t ok, pad;
  };
  static_assert(sizeof(Msg) % 8 == 0, "exchange record");
  Msg mine{};
  void* buf = nullptr;
  // uncached device memory where the runtime offers it (its accesses bypass the caches of every
  // agent, as RCCL's flags); else ordinary device memory (the accesses are system-scope atomics)
  if (hipExtMallocWithFlags(&buf, bytes, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    buf = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess) {
      (void)hipGetLastError();
      buf = nullptr;
    }
  }
  mine.ok = buf && hipMemset(buf, 0, bytes) == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
            hipIpcGetMemHandle(&mine.hdl, buf) == hipSuccess;
  if (!mine.ok) (void)hipGetLastError();
  Msg* dsend = nullptr;
  Msg* drecv = nullptr;
  std::vector<Msg> all(R);
  auto cleanup = [&] {
    if (dsend) (void)hipFree(dsend);
    if (drecv) (void)hipFree(drecv);
    dsend = drecv = nullptr;
  };
  LOAM_HIP(hipMalloc(&dsend, sizeof(Msg)));
  if (hipMalloc(&drecv, sizeof(Msg) * R) != hipSuccess) {
    cleanup();
    return LOAM_ERR_HIP;
  }
  auto exchange = [&]() -> int32_t {  // mine -> all (every rank's, in rank order)
    if (hipMemcpy(dsend, &mine, sizeof(Msg), hipMemcpyHostToDevice) != hipSuccess) return LOAM_ERR_HIP;
    TRY(comm_allgather(c, dsend, drecv, (int64_t)sizeof(Msg), h->st));
    if (hipStreamSynchronize(h->st) != hipSuccess ||
        hipMemcpy(all.data(), drecv, sizeof(Msg) * R, hipMemcpyDeviceToHost) != hipSuccess)
      return LOAM_ERR_HIP;
    return LOAM_OK;
  };
  int32_t rc = exchange();
  bool ok = rc == LOAM_OK;
  for (int r = 0; r < R && ok; ++r) ok = all[r].ok != 0;
  std::vector<unsigned long long> tab(2 * (size_t)R, 0ull);
  if (ok) {  // map the others' buffers; then agree that every rank mapped every buffer
    for (int r = 0; r < R; ++r) {
      void* p = buf;
      if (r != me) {
        p = nullptr;
        if (hipIpcOpenMemHandle(&p, all[r].hdl, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
          (void)hipGetLastError();
          p = nullptr;
        } else {
          h->ipc_open.push_back(p);
        }
      }
      tab[r] = reinterpret_cast<unsigned long long>(p);
      tab[R + r] = p ? reinterpret_cast<unsigned long long>(static_cast<char*>(p) + nslot * sizeof(double)) : 0ull;
      if (!p) ok = false;
    }
    const hipIpcMemHandle_t keep = mine.hdl;
    mine = Msg{};
    mine.hdl = keep;
    mine.ok = ok ? 1 : 0;
    if (rc == LOAM_OK) rc = exchange();
    ok = rc == LOAM_OK;
    for (int r = 0; r < R && ok; ++r) ok = all[r].ok != 0;
  }
  cleanup();
  if (!ok) {  // every rank arrives here alike: the two-kernel path
    for (void* p : h->ipc_open) (void)hipIpcCloseMemHandle(p);
    h->ipc_open.clear();
    if (buf) (void)hipFree(buf);
    return rc;
  }
  h->ipc_own = buf;
  unsigned long long* dtab = nullptr;
  const int32_t arc = dalloc(h, &dtab, tab.size());
  if (arc != LOAM_OK) return arc;
  // on the handle's stream, behind dalloc's zero fill there (a null-stream copy is not ordered
  // after it: the fill could land last and leave null peer pointers)
  LOAM_HIP(hipMemcpyAsync(dtab, tab.data(), sizeof(unsigned long long) * tab.size(), hipMemcpyHostToDevice, h->st));
  LOAM_HIP(hipStreamSynchronize(h->st));
  D.ipc_tab = dtab;
  D.ipc_B = (int)B;
  return LOAM_OK;
}

static int32_t mapper_create(const loam_params* p, int32_t device, int32_t n_streams, loam_comm* comm,
                             loam_mapper** out) {
  if (!out || n_streams <= 0) {
    set_error("loam_mapper_create: bad arguments");
    return LOAM_ERR_ARG;
  }
  *out = nullptr;
  TRY(ensure_device(device));
  LOAM_HIP(hipSetDevice(device));
  vh_spin_limit_from_env(device);
  lm_peer_spin_limit_from_env(device);
  auto* h = new loam_mapper;
  if (p) h->P = *p; else loam_params_default(&h->P);
  h->dev = device;
  h->B = n_streams;
  h->comm = comm;
  MapperDev& D = h->D;
  D.B = n_streams;
  if (comm) {
    D.sharded = 1;
    D.rank = comm->rank;
    D.nrank = comm->size;
  }
  D.max_in = h->P.max_input_points;
  D.map_cap = h->P.max_map_points;
  D.sub_cap = h->P.max_submap_points;
  D.scratch_cap = D.sub_cap + D.max_in;
  {
    const uint64_t cap = (uint64_t)D.map_cap, margin = (uint64_t)D.sub_cap + 2ull * D.max_in;
    h->compact_at = (uint32_t)std::max<uint64_t>(cap / 2, cap > margin ? cap - margin : 0);
    D.compact_at = h->compact_at;
    D.compact_due_at = h->compact_at;
  }
  D.max_chunks = LM_EBLK;
  {
    // k_lm_round: G workgroups per stream, B * G <= CUs x blocks/CU so that one launch fits the
    // GPU (speed only: the shares are claimed by whichever workgroups run, lm.h, so handles
    // sharing the GPU cannot deadlock).  LOAM_LM_PERSISTENT=0 selects the two-kernel path
    // (tests cover both).
    int occ = 0, cus = 0;
    const char* env = std::getenv("LOAM_LM_PERSISTENT");
    const bool allow = !(env && env[0] == '0');
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0)
      h->n_cu = cus;
    // sharded over several ranks: ranks of one process (loam_comm_create_local) meet inside the
    // persistent round (peer slots, lm.h); other transports all-reduce between two kernels per
    // pass.  At one rank every collective is the identity and the round stays one launch.
    const bool peer = comm && comm->size > 1 && comm->kind == 2;
    // ranks in separate processes: the same persistent round, meeting in IPC-mapped peer buffers
    // (ipc_peer_setup, below, once the stream exists; LOAM_PEER_LM=0 keeps the two-kernel path)
    const char* ienv = std::getenv("LOAM_PEER_LM");
    const bool ipc = comm && comm->size > 1 && comm->kind != 2 && !(ienv && ienv[0] == '0');
    h->want_ipc = false;
    if (allow && (!comm || comm->size == 1 || peer || ipc) &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_lm_round, LM_THREADS, 0) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess) {
      // 256 threads x 256 VGPRs: exactly one block per CU; the API can over-report by one
      // block per CU at some SGPR counts (MI355X_MICROARCH.md, correctness boundaries)
      occ = std::min(occ, 1);
      const int cap = occ * cus;
      // 16 at one stream: LM pass 26.5k -> 24.9k cycles once the leader loads the share partials
      // 8 at a time (4 / 8 / 12 / 16: 30.8k / 26.5k / 25.6k / 24.9k, tools/dbg_lm.py)
      // (with peer ranks on this device every rank's round must fit at once: a leader waits for
      // the other ranks' leaders)
      h->lm_G = std::min(LM_EBLK, std::min(16, cap / (peer ? lm_padded(n_streams) * comm->size : n_streams)));
      const char* genv = std::getenv("LOAM_LM_G");  // measurement override
      if (genv && std::atoi(genv) > 0) h->lm_G = std::min(LM_EBLK, std::atoi(genv));
      // cross-process ranks: every rank's leaders wait for each other; they fit even if every rank
      // shared this device (the test's two processes on one GPU); the members are claimed (lm.h)
      if (ipc && h->lm_G > 0) {
        if (lm_padded(n_streams) * comm->size <= cap) h->want_ipc = true;
        else h->lm_G = 0;
      }
      if (peer && h->lm_G > 0) {
        const size_t nd = (size_t)2 * n_streams * 2 * comm->size * LM_MAX_PASSES * LM_NACC;
        void* pb = nullptr;
        // the leaders (R x Bp) reserved against the device's LM capacity with every other group of
        // this process: all of them must fit at once (comm.hip); else the two-kernel path
        if (comm_peer_buffer(comm, nd * sizeof(double) + (size_t)n_streams * 2 * comm->size * sizeof(uint32_t),
                             lm_padded(n_streams) * comm->size, cap, &pb) == LOAM_OK) {
          D.lm_peer = static_cast<double*>(pb);
          D.lm_peer_flag = reinterpret_cast<uint32_t*>(D.lm_peer + nd);
        } else {
          h->lm_G = 0;  // the two-kernel path
        }
      }
    }
  }
  D.pcl_order = h->P.exact_voxel_order ? 1 : 0;
  // few streams: the input-order stack VoxelGrid over 8 workgroups per (stream, map)
  // (k_stack_part; 4 / 6 / 12 ranges measured slower)
  D.stack_k = (n_streams <= 4 && !D.pcl_order) ? 8 : 0;
  if (const char* kenv = std::getenv("LOAM_STACK_K"))  // measurement override (parts per stack)
    if (D.stack_k) D.stack_k = std::max(1, std::min(STACK_K_MAX, std::atoi(kenv)));
  D.leaf[0] = (float)h->P.mapping_line_resolution;
  D.leaf[1] = (float)h->P.mapping_plane_resolution;
  const size_t B = n_streams;
  auto fail = [&](int32_t rc) {
    free_all(h);
    delete h;
    return rc;
  };
  int32_t rc = LOAM_OK;
#define ALLOC(ptr, n) \
  if ((rc = dalloc(h, &(ptr), (n))) != LOAM_OK) return fail(rc)
  if (hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking) != hipSuccess) return fail(LOAM_ERR_HIP);
  if (hipStreamCreateWithFlags(&h->st2, hipStreamNonBlocking) != hipSuccess) return fail(LOAM_ERR_HIP);
  if (hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming) != hipSuccess)
    return fail(LOAM_ERR_HIP);
  for (auto& e : h->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(LOAM_ERR_HIP);
  if (hipEventCreateWithFlags(&h->ev_stack, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_sin[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&h->ev_sin[1], hipEventDisableTiming) != hipSuccess)
    return fail(LOAM_ERR_HIP);
  for (auto& ep : h->ev_fr)
    for (auto& e : ep)
      if (hipEventCreate(&e) != hipSuccess) return fail(LOAM_ERR_HIP);
  {
    const char* denv = std::getenv("LOAM_DEFER_EVERY");  // tests: force the deferral path
    D.defer_every = denv ? std::max(0, std::atoi(denv)) : 0;
  }
  // graphs pay off where launch gaps are the cost (B = 1: 0.750 -> 0.733 ms per frame); with
  // two handles of 64 streams, graph launches measured 20% slower (375k vs 470k iterations/s)
  h->use_graph = n_streams <= 4 ? 1 : 0;
  // cell split at few streams: B = 1 correspondence search 67.8 -> 35.6 us per round (8 lanes;
  // 4 lanes 43.4, 16 lanes 41.3, 2 lanes per query splitting the points 0.19 ms per frame); at
  // B = 128 it costs 1.2x (more lanes idle on pruned cells): one lane per query there
  h->knn_cs = n_streams <= 4 ? 8 : 0;
  D.knn_blk = n_streams <= 4 ? 4 * CORR_BLK : CORR_BLK;
  if (const char* benv = std::getenv("LOAM_KNN_BLK"))  // measurement override (cell-split workgroups per stream)
    if (h->knn_cs) D.knn_blk = std::max(1, std::min(64 * CORR_BLK, std::atoi(benv)));
  ALLOC(D.fr, B);
  for (int m = 0; m < 2; ++m) {
    ALLOC(D.in_pts[m], B * D.max_in);
    for (int p = 0; p < 2; ++p) ALLOC(h->stack_buf[p][m], B * D.max_in);
    D.stack[m] = h->stack_buf[0][m];
  }
  ALLOC(D.arena, B * 2 * 2 * (size_t)D.map_cap);
  ALLOC(D.carena, B * 2 * 2 * (size_t)D.map_cap);
  ALLOC(D.ctab, B * 2 * 2 * 4 * (size_t)D.map_cap);
  ALLOC(h->cube_tab[0], B * 2 * NCUBE);
  ALLOC(h->cube_tab[1], B * 2 * NCUBE);
  ALLOC(D.extra_flag, B * 2 * NCUBE);
  D.knn_stride = B * 2 * (size_t)D.max_in;
  ALLOC(D.knn_id, 5 * D.knn_stride);
  ALLOC(D.r_type, B * 2 * (size_t)D.max_in);
  ALLOC(D.r_px, B * 2 * (size_t)D.max_in);
  ALLOC(D.r_py, B * 2 * (size_t)D.max_in);
  ALLOC(D.r_pz, B * 2 * (size_t)D.max_in);
  for (int k = 0; k < 3; ++k) {
    ALLOC(D.r_a[k], B * 2 * (size_t)D.max_in);
    ALLOC(D.r_b[k], B * 2 * (size_t)D.max_in);
  }
  ALLOC(D.ins_pts, B * 2 * (size_t)D.max_in);
  ALLOC(D.ins_tag, B * 2 * (size_t)D.max_in);
  ALLOC(D.ins_sorted, B * 2 * (size_t)D.max_in);
  ALLOC(D.ins_off, B * 2 * (size_t)(INS_SLOTS + 1));
  ALLOC(D.stable_tok, B * 2 * (size_t)NCUBE);
  ALLOC(h->tok_tmp, B * 2 * (size_t)NCUBE);
  ALLOC(D.dbg, LOAM_DEBUG_COUNTERS);
  {  // phase cycle counters (readcyclecounter + device-scope atomics in the kernels): diagnostics only
    const char* penv = std::getenv("LOAM_PHASE_COUNTERS");
    D.pdbg = (penv && std::atoi(penv) > 0) ? D.dbg : nullptr;
  }
  ALLOC(D.vx_pts, B * 2 * (size_t)D.scratch_cap);
  if (D.pcl_order) {
    const size_t ps = mp_scratch(D);
    ALLOC(D.pe, B * 2 * ps);
    ALLOC(D.pa, B * 2 * ps);
    ALLOC(D.pb, B * 2 * ps);
    ALLOC(D.ps, B * 2 * ps);
    ALLOC(D.pseg, B * 2 * (9 * (ps / 16) + 9));
  }
  ALLOC(D.vx_idx, B * 2 * (size_t)D.scratch_cap);
  ALLOC(D.stk_part, B * 2 * (size_t)STACK_K_MAX);
  for (int p = 0; p < 2; ++p) {
    ALLOC(h->stk_n_buf[p], B * 2);
    ALLOC(h->stk_err_buf[p], B);
    // few streams: the stack inputs in page-locked host memory the stack kernels read in place
    // (mapped), no H2D copy ahead of the stack VoxelGrid, which heads the blocking frame's critical
    // path; many streams: a device copy (256 workgroups reading host memory cost the stack family
    // ~0.05 ms per step at B = 128, profiles/r6_member_chunks_ab.txt)
    if (B <= 4) {
      void* dp = nullptr;
      if (!h->hsin[p].assign(B, StackIn{}, hipHostMallocMapped | hipHostMallocCoherent) ||
          hipHostGetDevicePointer(&dp, h->hsin[p].data(), 0) != hipSuccess)
        return fail(LOAM_ERR_HIP);
      h->sin_buf[p] = static_cast<StackIn*>(dp);
    } else {
      ALLOC(h->sin_buf[p], B);
      if (!h->hsin[p].assign(B, StackIn{})) return fail(LOAM_ERR_HIP);
    }
  }
  D.sin = h->sin_buf[0];
  D.stk_n = h->stk_n_buf[0];
  D.stk_err = h->stk_err_buf[0];
  ALLOC(h->d_stk_ready, 2);
  ALLOC(D.stk_pts, B * 2 * (size_t)D.max_in);
  ALLOC(D.stk_idx, B * 2 * (size_t)D.max_in);
  ALLOC(D.partials, B * (size_t)D.max_chunks * LM_NACC);
  ALLOC(D.lm_sync, B * 2 * LM_SYNC_WORDS);
  ALLOC(D.lm_xpub, B * 2 * 8);
  ALLOC(D.tickets, B);
  ALLOC(D.lm_tick, B);
  D.rq_cap = B * 2 * INS_SLOTS;
  ALLOC(D.rq, (size_t)RQ_CLASSES * D.rq_cap);
  ALLOC(D.rq_ctl, RQ_CLASSES);
  ALLOC(h->d_map_off, 2 * NCUBE + 1);
  ALLOC(h->d_new_off, B * 2 * (NCUBE + 1));
  if (D.sharded) {
    for (int m = 0; m < 2; ++m) D.blk_v[m] = shard_block_voxels(D.leaf[m]);
    const size_t nq = B * 2 * (size_t)D.max_in;
    NnRec* recv = nullptr;
    ALLOC(D.wcnt, B * 2 * (size_t)WIN_MAX);
    ALLOC(D.nn_send, nq);
    if (D.nrank > 1) {
      ALLOC(recv, nq * D.nrank);
      D.nn_recv = recv;
    } else {
      D.nn_recv = D.nn_send;  // one rank: the all-gather is the identity
    }
    ALLOC(D.nn_xyz, 5 * nq);
    ALLOC(D.lm_red, B * (size_t)LM_NACC);
    ALLOC(D.pose_x, (size_t)D.nrank * B * 8);
    ALLOC(h->d_q_off, B + 1);
    D.q_off = h->d_q_off;
    if (!h->q_off.assign(2 * (B + 1), 0)) return fail(LOAM_ERR_HIP);  // [parity][B + 1]
    if (D.nrank == 1) {  // fixed query slots: no per-frame host read of the stack sizes
      for (size_t s = 0; s <= B; ++s) h->q_off[s] = (int)(s * 2 * (size_t)D.max_in);
      if (hipMemcpyAsync(h->d_q_off, h->q_off.data(), sizeof(int) * (B + 1), hipMemcpyHostToDevice, h->st) !=
          hipSuccess)
        return fail(LOAM_ERR_HIP);
    }
  }
#undef ALLOC
  D.cube_tab = h->cube_tab[0];
  if (!h->hf.assign(B, StreamFrame{})) return fail(LOAM_ERR_HIP);
  for (int p = 0; p < 2; ++p) {
    void* dp = nullptr;
    if (!h->hfo[p].assign(B, StreamFrame{}, hipHostMallocMapped | hipHostMallocCoherent) ||
        !h->fin[p].assign(B, FrameIn{}, hipHostMallocMapped | hipHostMallocCoherent) ||
        hipHostGetDevicePointer(&dp, h->fin[p].data(), 0) != hipSuccess)
      return fail(LOAM_ERR_HIP);
    h->fin_dev[p] = reinterpret_cast<const FrameIn*>(dp);
    if (hipHostGetDevicePointer(&dp, h->hfo[p].data(), 0) != hipSuccess) return fail(LOAM_ERR_HIP);
    h->hfo_dev[p] = reinterpret_cast<StreamFrame*>(dp);
  }
  {
    void* dp = nullptr;
    if (!h->done.assign(2, 0ull, hipHostMallocMapped | hipHostMallocCoherent) ||
        hipHostGetDevicePointer(&dp, h->done.data(), 0) != hipSuccess)
      return fail(LOAM_ERR_HIP);
    h->done_dev = reinterpret_cast<unsigned long long*>(dp);
    if (!h->done_early.assign(2, 0ull, hipHostMallocMapped | hipHostMallocCoherent) ||
        hipHostGetDevicePointer(&dp, h->done_early.data(), 0) != hipSuccess)
      return fail(LOAM_ERR_HIP);
    h->done_early_dev = reinterpret_cast<unsigned long long*>(dp);
    for (int p = 0; p < 2; ++p) {
      if (!h->hfo_early[p].assign(B, StreamFrame{}, hipHostMallocMapped | hipHostMallocCoherent) ||
          hipHostGetDevicePointer(&dp, h->hfo_early[p].data(), 0) != hipSuccess)
        return fail(LOAM_ERR_HIP);
      h->hfo_early_dev[p] = reinterpret_cast<StreamFrame*>(dp);
    }
  }
  h->hs.assign(B, HostStream{});
  h->last_tail.assign(B, std::array<uint32_t, 2>{0u, 0u});
  for (size_t s = 0; s < B; ++s) {
    StreamFrame& F = h->hf[s];
    F.cen[0] = 10; F.cen[1] = 10; F.cen[2] = 5;
    F.pose[3] = F.wodom[3] = F.wmap[3] = 1.0;
  }
  if (hipStreamSynchronize(h->st) != hipSuccess) return fail(LOAM_ERR_HIP);  // zero-fills done
  if (h->want_ipc) {  // collective: every rank of the comm creates its mapper
    if ((rc = ipc_peer_setup(h)) != LOAM_OK) return fail(rc);
    if (!D.ipc_tab) h->lm_G = 0;  // some rank could not map the buffers: the two-kernel path
  }
  *out = h;
  return LOAM_OK;
}

int32_t loam_mapper_create(const loam_params* p, int32_t device, int32_t n_streams, loam_mapper** out) {
  return mapper_create(p, device, n_streams, nullptr, out);
}

int32_t loam_mapper_create_sharded(const loam_params* p, int32_t device, int32_t n_streams, loam_comm* comm,
                                   loam_mapper** out) {
  if (!comm) {
    set_error("loam_mapper_create_sharded: null comm");
    return LOAM_ERR_ARG;
  }
  return mapper_create(p, device, n_streams, comm, out);
}

int32_t loam_shard_owner(const float* xyz, float leaf, int32_t nrank) {
  if (!xyz || !(leaf > 0.f) || nrank < 1) return LOAM_ERR_ARG;
  return shard_owner(xyz[0], xyz[1], xyz[2], 1.0f / leaf, shard_block_voxels(leaf), nrank);
}

static int32_t finish_oldest(loam_mapper* h);
static int32_t settle_all(loam_mapper* h);
static bool chain_capable(const loam_mapper* h);
// every frame in flight is finished before anything reads or changes the handle's state
#define SETTLE(h)                                \
  do {                                           \
    if ((h) && !(h)->q.empty()) {                \
      LOAM_HIP(hipSetDevice((h)->dev));          \
      TRY(settle_all(h));                        \
    }                                            \
  } while (0)
// the result calls (pose, stats, state, iterations) report the newest finished frame: they finish
// the oldest frame in the queue unless it was given behind another (whose results they report)
#define SETTLE_RESULTS(h)                                                                   \
  do {                                                                                      \
    if ((h) && !(h)->q.empty() && !(h)->q.front().behind && !(h)->q.front().early_seen) { \
      LOAM_HIP(hipSetDevice((h)->dev));                                                     \
      TRY(finish_oldest(h));                                                                \
    }                                                                                       \
  } while (0)

int32_t loam_mapper_destroy(loam_mapper* h) {
  if (!h) return LOAM_ERR_ARG;
  (void)hipSetDevice(h->dev);
  while (!h->q.empty()) (void)finish_oldest(h);
  (void)hipStreamSynchronize(h->st);
  (void)hipStreamSynchronize(h->st2);
  free_all(h);
  delete h;
  return LOAM_OK;
}

int32_t loam_mapper_reset(loam_mapper* h) {
  if (!h) return LOAM_ERR_ARG;
  SETTLE(h);
  LOAM_HIP(hipSetDevice(h->dev));
  LOAM_HIP(hipStreamSynchronize(h->st2));  // stacks queued ahead are dropped with their inputs
  for (int p = 0; p < 2; ++p)
    LOAM_HIP(hipMemsetAsync(h->cube_tab[p], 0, sizeof(uint2) * h->B * 2 * NCUBE, h->st));
  LOAM_HIP(hipMemsetAsync(h->D.stable_tok, 0, sizeof(uint32_t) * h->B * 2 * NCUBE, h->st));
  LOAM_HIP(hipStreamSynchronize(h->st));
  for (int s = 0; s < h->B; ++s) {
    h->hf[s] = StreamFrame{};
    h->hf[s].cen[0] = 10; h->hf[s].cen[1] = 10; h->hf[s].cen[2] = 5;
    h->hf[s].pose[3] = h->hf[s].wodom[3] = h->hf[s].wmap[3] = 1.0;
    h->last_tail[s] = {0u, 0u};
    h->hs[s] = HostStream{};
  }
  return LOAM_OK;
}

// LaserMapping::input (laser_mapping.cpp:178-209): the clouds and odometry pose of the next
// solve.  Kept apart from a frame in flight (loam_mapper_solve_async): the solve that takes it
// computes the initial guess (:206-207) once the previous frame's transformUpdate is known.
static int32_t mapper_input_common(loam_mapper* h, int32_t s, const float* corner, int32_t nc,
                                   const float* surf, int32_t ns, const double* q_wodom,
                                   const double* t_wodom, int32_t skip, hipMemcpyKind kind) {
  TRY(check_stream(h, s));
  if (!q_wodom || !t_wodom || nc < 0 || ns < 0 || (nc > 0 && !corner) || (ns > 0 && !surf)) {
    set_error("loam_mapper_input: bad arguments");
    return LOAM_ERR_ARG;
  }
  if (nc > h->D.max_in || ns > h->D.max_in) {
    set_error("loam_mapper_input: cloud larger than max_input_points");
    return LOAM_ERR_CAPACITY;
  }
  LOAM_HIP(hipSetDevice(h->dev));
  HostStream& H = h->hs[s];
  if (skip) {  // laser_mapping.cpp:197-201: high-frequency pose only (needs the last transformUpdate)
    SETTLE(h);
    for (int i = 0; i < 4; ++i) H.q_wodom[i] = q_wodom[i];
    for (int i = 0; i < 3; ++i) H.t_wodom[i] = t_wodom[i];
    H.skip = true;
    double pose[7];
    host_initial_guess(H, pose);
    for (int i = 0; i < 4; ++i) H.q_hf[i] = pose[i];
    for (int i = 0; i < 3; ++i) H.t_hf[i] = pose[4 + i];
    H.in_ready = false;
    H.stk_launched = false;
    return LOAM_OK;
  }
  if (kind == hipMemcpyHostToDevice) {
    // LaserMapping::input deep-copies the clouds (:188-190); on the stack stream, after any
    // stack still reading the staging buffer
    H.in_p[0] = h->D.in_pts[0] + (size_t)s * h->D.max_in;
    H.in_p[1] = h->D.in_pts[1] + (size_t)s * h->D.max_in;
    if (nc) LOAM_HIP(hipMemcpyAsync((void*)H.in_p[0], corner, sizeof(float4) * nc, kind, h->st2));
    if (ns) LOAM_HIP(hipMemcpyAsync((void*)H.in_p[1], surf, sizeof(float4) * ns, kind, h->st2));
  } else {
    // HBM-resident clouds are read in place: they must stay valid until the stack VoxelGrid has
    // read them (loam_mapper_solve returns, or the wait after loam_mapper_solve_async)
    H.in_p[0] = reinterpret_cast<const float4*>(corner);
    H.in_p[1] = reinterpret_cast<const float4*>(surf);
  }
  H.in_n[0] = nc;
  H.in_n[1] = ns;
  for (int i = 0; i < 4; ++i) H.in_q[i] = q_wodom[i];
  for (int i = 0; i < 3; ++i) H.in_t[i] = t_wodom[i];
  H.skip = false;
  H.in_ready = true;
  H.stk_launched = false;
  return LOAM_OK;
}

int32_t loam_mapper_input(loam_mapper* h, int32_t s, const float* corner, int32_t nc, const float* surf,
                          int32_t ns, const double* q_wodom, const double* t_wodom, int32_t skip) {
  return mapper_input_common(h, s, corner, nc, surf, ns, q_wodom, t_wodom, skip, hipMemcpyHostToDevice);
}

int32_t loam_mapper_input_device(loam_mapper* h, int32_t s, const float* corner, int32_t nc,
                                 const float* surf, int32_t ns, const double* q_wodom,
                                 const double* t_wodom, int32_t skip) {
  return mapper_input_common(h, s, corner, nc, surf, ns, q_wodom, t_wodom, skip, hipMemcpyDeviceToDevice);
}

// HIP events around each launch when profiling is on (accumulated per kernel family)
static hipError_t prof_begin(loam_mapper* h, int fam, hipEvent_t* stop, hipStream_t st) {
  *stop = nullptr;
  if (!h->prof) return hipSuccess;
  size_t k = h->ev_fam.size() * 2;
  while (h->ev_pool.size() < k + 2) {
    hipEvent_t e;
    hipError_t err = hipEventCreate(&e);
    if (err != hipSuccess) return err;
    h->ev_pool.push_back(e);
  }
  h->ev_fam.push_back(fam);
  *stop = h->ev_pool[k + 1];
  return hipEventRecord(h->ev_pool[k], st);
}
// the stop event of a timed launch: recorded by end(), or, when the launch body returns early (a
// TRY inside it), by the destructor, so no listed (start, stop) pair is left without its stop
struct ProfStop {
  hipEvent_t ev = nullptr;
  hipStream_t st = nullptr;
  hipError_t end() {
    const hipError_t e = ev ? hipEventRecord(ev, st) : hipSuccess;
    ev = nullptr;
    return e;
  }
  ~ProfStop() { (void)end(); }
};
#define LAUNCH_ON(stream, fam, ...)                     \
  do {                                                  \
    ProfStop stop_;                                     \
    stop_.st = (stream);                                \
    LOAM_HIP(prof_begin(h, (fam), &stop_.ev, (stream))); \
    __VA_ARGS__;                                        \
    LOAM_HIP(stop_.end());                              \
  } while (0)
#define LAUNCH(fam, ...) LAUNCH_ON(h->st, fam, __VA_ARGS__)

int32_t loam_mapper_input_device_batch(loam_mapper* h, int32_t n, const int32_t* streams,
                                       const uint64_t* d_corner, const int32_t* n_corner,
                                       const uint64_t* d_surf, const int32_t* n_surf,
                                       const double* q_wodom, const double* t_wodom) {
  if (!h || n < 0 || (n > 0 && (!streams || !d_corner || !n_corner || !d_surf || !n_surf || !q_wodom || !t_wodom))) {
    set_error("loam_mapper_input_device_batch: bad arguments");
    return LOAM_ERR_ARG;
  }
  for (int i = 0; i < n; ++i) {
    int32_t rc = mapper_input_common(h, streams[i], reinterpret_cast<const float*>(d_corner[i]), n_corner[i],
                                     reinterpret_cast<const float*>(d_surf[i]), n_surf[i], q_wodom + 4 * i,
                                     t_wodom + 3 * i, 0, hipMemcpyDeviceToDevice);
    if (rc != LOAM_OK) return rc;
  }
  return LOAM_OK;
}

int32_t loam_mapper_lm_path(loam_mapper* h) {
  if (!h) return LOAM_ERR_ARG;
  if (h->lm_G <= 0) return 0;
  if (h->D.lm_peer) return 2;
  if (h->D.ipc_tab) return 3;
  return 1;
}

int64_t loam_mapper_total_iterations(loam_mapper* h) {
  if (!h) return LOAM_ERR_ARG;
  SETTLE_RESULTS(h);
  int64_t it = 0;
  for (int s = 0; s < h->B; ++s)
    if (h->hs[s].solved_last) it += h->hs[s].st.lm[0].iterations + h->hs[s].st.lm[1].iterations;
  return it;
}

int32_t loam_mapper_stats_all(loam_mapper* h, loam_map_stats* out, int32_t n) {
  SETTLE_RESULTS(h);
  if (!h || !out || n < 0 || n > h->B) return LOAM_ERR_ARG;
  for (int s = 0; s < n; ++s) out[s] = h->hs[s].st;
  return LOAM_OK;
}

// The stack VoxelGrids (laser_mapping.cpp:492-500) of every stream whose input has none queued
// yet, in one launch on the stack stream, into the stack buffers of the next frame's parity.
// They read only the frame's body-frame input, so they may run beside a frame in flight.
static int32_t launch_stacks(loam_mapper* h) {
  const int par = h->spar, B = h->B;
  for (const FrameRec& R : h->q)  // that parity's stack buffers still belong to a frame in flight
    if (R.fpar == par) return LOAM_OK;
  bool any = false;
  LOAM_HIP(hipEventSynchronize(h->ev_sin[par]));  // the last reads of hsin[par] are done
  StackIn* in = h->hsin[par].data();
  for (int s = 0; s < B; ++s) {
    HostStream& H = h->hs[s];
    const bool go = H.in_ready && !H.stk_launched;
    in[s].active = go ? 1 : 0;
    if (!go) continue;
    any = true;
    H.stk_launched = true;
    H.stk_seq = h->stack_seq + 1;
    for (int m = 0; m < 2; ++m) {
      in[s].p[m] = H.in_p[m];
      in[s].n[m] = H.in_n[m];
    }
  }
  if (!any) return LOAM_OK;
  const unsigned long long seq = ++h->stack_seq;
  MapperDev D = h->D;
  D.sin = h->sin_buf[par];
  D.stk_n = h->stk_n_buf[par];
  D.stk_err = h->stk_err_buf[par];
  for (int m = 0; m < 2; ++m) D.stack[m] = h->stack_buf[par][m];
  hipStream_t s2 = h->st2;
  if (h->B > 4) LOAM_HIP(hipMemcpyAsync(h->sin_buf[par], in, sizeof(StackIn) * B, hipMemcpyHostToDevice, s2));
  if (D.stack_k) {
    LAUNCH_ON(s2, FAM_STACK, k_stack_part<<<B * 2 * D.stack_k, VX_THREADS, 0, s2>>>(D));
    LAUNCH_ON(s2, FAM_STACK, k_stack_cat<<<B * 2, VX_THREADS, 0, s2>>>(D));
  } else {
    if (D.pcl_order) LAUNCH_ON(s2, FAM_STACK, k_stack_ds<true><<<B * 2, VX_THREADS, 0, s2>>>(D));
    else LAUNCH_ON(s2, FAM_STACK, k_stack_ds<false><<<B * 2, VX_THREADS, 0, s2>>>(D));
  }
  k_stack_done<<<1, 64, 0, s2>>>(h->d_stk_ready + par, seq);
  LOAM_HIP(hipGetLastError());
  LOAM_HIP(hipEventRecord(h->ev_sin[par], s2));  // (hsin[par] is read, in place or by the copy, until here)
  LOAM_HIP(hipEventRecord(h->ev_stack, s2));
  return LOAM_OK;
}

int32_t loam_mapper_prefetch(loam_mapper* h) {
  if (!h) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  return launch_stacks(h);
}

// k_revox workgroups: one per possible item
static int revox_grid(const loam_mapper* h) { return h->B * 2 * INS_SLOTS; }
// the frame's re-VoxelGrid
static void launch_revox(const loam_mapper* h, const MapperDev& D, hipStream_t st) {
  if (D.pcl_order) k_revox<true><<<revox_grid(h), VX_THREADS, 0, st>>>(D);
  else k_revox<false><<<revox_grid(h), VX_THREADS, 0, st>>>(D);
}

// the frame's kernel sequence for the hipGraph path: k_frame_prep (records of a queued frame,
// stack sizes, submap offsets), 2 x (kNN, geometry, LM round), insertion, re-VoxelGrid, and the
// records back to the D2H buffer of the frame's stack parity.  Every kernel argument is fixed per
// (cube-table parity, stack parity): the frame's values travel in the records and FrameIn.
static void capture_frame(loam_mapper* h, const MapperDev& D, int fpar, hipStream_t st) {
  const int B = h->B;
  k_frame_prep<<<B, 128, 0, st>>>(D);
  for (int round = 0; round < 2; ++round) {
    if (h->knn_cs) k_knn<8, true><<<B * D.knn_blk, CORR_THREADS, 0, st>>>(D, round);
    else k_knn<1><<<B * CORR_BLK, CORR_THREADS, 0, st>>>(D, round);
    k_geom<<<B * CORR_BLK, CORR_THREADS, 0, st>>>(D, round);
    k_lm_round<<<lm_padded(B) * h->lm_G, LM_THREADS, 0, st>>>(D, round, h->lm_G);
  }
  // (loam_mapper_solve_pose) the final poses and the frame's stats are in the records now
  if (h->early) k_frame_out<<<1, 256, 0, st>>>(D, h->hfo_early_dev[fpar], h->done_early_dev + fpar);
  k_insert_bucket<<<B * 2, VX_THREADS, 0, st>>>(D);
  launch_revox(h, D, st);
  k_frame_out<<<1, 256, 0, st>>>(D, h->hfo_dev[fpar], h->done_dev + fpar);
}

// Enqueue one solveMapping of every stream with an input (the work of loam_mapper_solve up to
// the host bookkeeping, which mapper_finish_rec does).  chained: queued behind the frame in
// flight, whose results the host does not have yet: the device prepares the stream records
// (k_frame_prep) from what that frame left, and only the graph path runs.
static int32_t mapper_enqueue(loam_mapper* h, bool chained, FrameRec& R) {
  MapperDev& D = h->D;
  const int B = h->B;
  TRY(launch_stacks(h));  // inputs not prefetched
  const int fpar = h->spar;  // the stack parity of this frame
  D.sin = h->sin_buf[fpar];
  D.stk_n = h->stk_n_buf[fpar];
  D.stk_err = h->stk_err_buf[fpar];
  D.fin = h->fin_dev[fpar];
  D.stk_ready = h->d_stk_ready + fpar;
  for (int m = 0; m < 2; ++m) D.stack[m] = h->stack_buf[fpar][m];
  R = FrameRec{};
  R.chained = chained;
  R.fpar = fpar;
  R.active.assign(B, 0);
  R.wodom.assign(B, std::array<double, 7>{0, 0, 0, 1, 0, 0, 0});
  R.in_p.assign(B, std::array<const float4*, 2>{nullptr, nullptr});
  R.in_n.assign(B, std::array<int, 2>{0, 0});
  R.stk_seq.assign(B, 0ull);
  bool any = false;
  for (int s = 0; s < B; ++s) {  // the inputs become the frame
    HostStream& H = h->hs[s];
    if (!H.in_ready) continue;
    if (!H.stk_launched) {
      set_error("loam_mapper: stack buffers of the frame's parity still in use");
      return LOAM_ERR_ARG;
    }
    any = true;
    R.active[s] = 1;
    for (int i = 0; i < 4; ++i) R.wodom[s][i] = H.in_q[i];
    for (int i = 0; i < 3; ++i) R.wodom[s][4 + i] = H.in_t[i];
    R.in_p[s] = {H.in_p[0], H.in_p[1]};
    R.in_n[s] = {H.in_n[0], H.in_n[1]};
    R.stk_seq[s] = H.stk_seq;
    H.in_ready = false;
    H.stk_launched = false;
  }
  if (!any) return LOAM_OK;
  R.seq = ++h->seq;
  h->frame_counter++;
  D.epoch = h->frame_counter;
  D.cube_tab = h->cube_tab[h->parity];
  hipStream_t st = h->st;
  FrameIn* fin = h->fin[fpar].data();
  if (chained) {
    for (int s = 0; s < B; ++s) {
      FrameIn& I = fin[s];
      I = FrameIn{};
      I.mode = 1;
      I.active = R.active[s];
      for (int i = 0; i < 7; ++i) I.wodom[i] = R.wodom[s][i];
      I.in_ptr[0] = R.in_p[s][0];
      I.in_ptr[1] = R.in_p[s][1];
      I.n[0] = R.in_n[s][0];
      I.n[1] = R.in_n[s][1];
      I.epoch = h->frame_counter;
      I.stack_seq = R.stk_seq[s];
    }
  } else {
    // the host prepares the records: initial guess (:206-207), centerCube + recentering
    // (:228-444), window (:455-472)
    for (int s = 0; s < B; ++s) {
      StreamFrame& F = h->hf[s];
      const HostStream& H = h->hs[s];
      frame_reset(F);
      F.active = R.active[s];
      if (!F.active) continue;  // (a stream deferred in a frame still in flight stays deferred)
      F.deferred = 0;
      for (int i = 0; i < 4; ++i) F.wmap[i] = H.q_wmap_wodom[i];
      for (int i = 0; i < 3; ++i) F.wmap[4 + i] = H.t_wmap_wodom[i];
      for (int i = 0; i < 7; ++i) F.wodom[i] = R.wodom[s][i];
      pose_initial_guess(F.wmap, F.wodom, F.pose);
      frame_center(F.pose, F.cen, F.center, F.shift);
      frame_window(F);
      F.epoch = h->frame_counter;
      F.in_ptr[0] = R.in_p[s][0];
      F.in_ptr[1] = R.in_p[s][1];
      F.nc_in = R.in_n[s][0];
      F.ns_in = R.in_n[s][1];
    }
    for (int s = 0; s < B; ++s) {  // mode 0: the records as uploaded
      fin[s] = FrameIn{};
      fin[s].epoch = h->frame_counter;
      fin[s].active = R.active[s];
      fin[s].stack_seq = R.stk_seq[s];
    }
  }
  bool any_shift = false;
  for (int s = 0; s < B && !chained; ++s)
    any_shift |= h->hf[s].active && (h->hf[s].shift[0] || h->hf[s].shift[1] || h->hf[s].shift[2]);
  // arenas past the compaction threshold are compacted ahead of this frame.  With frames queued
  // behind each other, a little early (the threshold less three frames' growth) so that queued
  // frames rarely meet a due compaction (they would be deferred); the moves are verbatim, the
  // results do not depend on when they happen.
  uint32_t due_at = h->compact_at;
  if (chain_capable(h)) {
    const uint64_t ahead = 3ull * h->grow_max + 4096ull;
    due_at = (uint32_t)std::max<uint64_t>(h->compact_at / 2, h->compact_at > ahead ? h->compact_at - ahead : 0);
  }
  // (a queued frame: the tails known now are those before the frame in flight, which may add
  // one frame's growth; the kernels test the tails as they are when they run)
  bool compact_due = false;
  const uint64_t unknown = chained ? (uint64_t)h->grow_max : 0ull;
  for (int s = 0; s < B && !compact_due; ++s)
    compact_due = h->hf[s].arena_tail[0] + unknown > due_at || h->hf[s].arena_tail[1] + unknown > due_at;
  const bool graph = chained || (h->use_graph && !h->prof && !any_shift && !D.sharded && h->lm_G > 0);
  R.graph = graph;
  if (graph) {
    hipGraphExec_t& ge = h->gexec[h->parity][fpar];
    // a frame queued behind the one in flight is launched kernel by kernel: a graph launch costs
    // 14 against 6 us between two frames at one stream (rocprofv3 trace); the others as the graph
    const bool direct = chained;
    if (!ge && !direct) {
      hipGraph_t gr = nullptr;
      LOAM_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      capture_frame(h, D, fpar, st);
      LOAM_HIP(hipStreamEndCapture(st, &gr));
      const hipError_t ie = hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0);
      (void)hipGraphDestroy(gr);
      LOAM_HIP(ie);
    }
    if (!chained) LOAM_HIP(hipMemcpyAsync(D.fr, h->hf.data(), sizeof(StreamFrame) * B, hipMemcpyHostToDevice, st));
    if (compact_due) {  // compactions ahead of the graph (a queued frame's k_frame_prep defers if still due)
      MapperDev Dc = D;
      Dc.compact_due_at = due_at;
      k_compact_scan<<<B * 2, VX_THREADS, 0, st>>>(Dc, h->d_new_off);
      k_compact_copy<<<dim3(128, B * 2), 256, 0, st>>>(Dc, h->d_new_off);
      k_compact_commit<<<B * 2, 256, 0, st>>>(Dc, h->d_new_off);
      LOAM_HIP(hipGetLastError());
    }
    // the frame's stacks: waited for by k_frame_prep on the device (stack_seq)
    // a queued frame is not timed: its start is its predecessor's end, and the timing markers
    // between two graph launches would cost the device time
    if (!chained) LOAM_HIP(hipEventRecord(h->ev_fr[fpar][0], st));
    if (direct) {
      capture_frame(h, D, fpar, st);
      LOAM_HIP(hipGetLastError());
    } else {
      LOAM_HIP(hipGraphLaunch(ge, st));
    }
    if (!chained) LOAM_HIP(hipEventRecord(h->ev_fr[fpar][1], st));
    R.epoch = h->frame_counter;
    h->spar ^= 1;  // the next frame's stacks go to the other buffers
    return LOAM_OK;
  }
  LOAM_HIP(hipMemcpyAsync(D.fr, h->hf.data(), sizeof(StreamFrame) * B, hipMemcpyHostToDevice, st));
  LOAM_HIP(hipEventRecord(h->ev_fr[fpar][0], st));
  // compaction queued ahead of this frame (each workgroup checks its own pair's tail against
  // due_at), so the host never waits on it
  if (compact_due) {
    MapperDev Dc = D;
    Dc.compact_due_at = due_at;
    k_compact_scan<<<B * 2, VX_THREADS, 0, st>>>(Dc, h->d_new_off);
    k_compact_copy<<<dim3(128, B * 2), 256, 0, st>>>(Dc, h->d_new_off);
    k_compact_commit<<<B * 2, 256, 0, st>>>(Dc, h->d_new_off);
    LOAM_HIP(hipGetLastError());
  }
  // the stack VoxelGrids run on the second stream (launch_stacks: at prefetch, or at the start
  // of this solve), overlapping the cube shift and submap preparation; joined before the
  // correspondences
  if (any_shift) {
    LAUNCH(FAM_OTHER, k_shift_cubes<<<dim3(16, B), 256, 0, st>>>(D, h->cube_tab[h->parity],
                                                                 h->cube_tab[1 - h->parity], h->tok_tmp));
    LOAM_HIP(hipMemcpyAsync(D.stable_tok, h->tok_tmp, sizeof(uint32_t) * B * 2 * NCUBE, hipMemcpyDeviceToDevice, st));
    h->parity ^= 1;
    D.cube_tab = h->cube_tab[h->parity];
  }
  const bool multi = D.sharded && D.nrank > 1;  // collectives that are not the identity
  if (D.sharded) {  // the submap sizes over all ranks
    LAUNCH(FAM_OTHER, k_submap_count<<<B, 256, 0, st>>>(D));
    if (multi) TRY(comm_allreduce(h->comm, D.wcnt, (int64_t)B * 2 * WIN_MAX, LOAM_DT_I32, st));
  }
  LAUNCH(FAM_OTHER, k_submap_prep<<<B, 128, 0, st>>>(D));
  LOAM_HIP(hipEventRecord(h->ev[1], st));
  LOAM_HIP(hipStreamWaitEvent(st, h->ev_stack, 0));
  LAUNCH(FAM_OTHER, k_stack_counts<<<B, 64, 0, st>>>(D));
  size_t q_tot = 0;
  if (multi) {
    // each stream's queries in the exchange: slots sized by the frame's input counts, which the
    // host has without waiting (a VoxelGrid never outputs more points than it reads, :492-500),
    // identical on every rank.  The host array is double-buffered by the frame parity: its copy
    // may still be queued when the next frame is enqueued.
    int* qo = h->q_off.data() + (size_t)fpar * (B + 1);
    for (int s = 0; s < B; ++s) {
      const StreamFrame& F = h->hf[s];
      qo[s] = (int)q_tot;
      if (F.active) q_tot += (size_t)F.nc_in + F.ns_in;
    }
    qo[B] = (int)q_tot;
    LOAM_HIP(hipMemcpyAsync(h->d_q_off, qo, sizeof(int) * (B + 1), hipMemcpyHostToDevice, st));
  }
  for (int round = 0; round < 2; ++round) {
    if (h->knn_cs) LAUNCH(FAM_CORR, (k_knn<8, true><<<B * D.knn_blk, CORR_THREADS, 0, st>>>(D, round)));
    else LAUNCH(FAM_CORR, k_knn<1><<<B * CORR_BLK, CORR_THREADS, 0, st>>>(D, round));
    if (D.sharded) {  // every rank's candidates -> the exact 5-NN on every rank
      if (multi)
        TRY(comm_allgather(h->comm, D.nn_send, const_cast<NnRec*>(D.nn_recv), (int64_t)(q_tot * sizeof(NnRec)), st));
      LAUNCH(FAM_CORR, k_nn_merge<<<B * CORR_BLK, CORR_THREADS, 0, st>>>(D));
    }
    LAUNCH(FAM_CORR, k_geom<<<B * CORR_BLK, CORR_THREADS, 0, st>>>(D, round));
    if (h->lm_G > 0) {
      if (D.lm_peer) {  // in-process ranks: one launch for every rank's round (k_lm_group)
        LmRankArgs a{D.fr, D.r_type, D.r_px, D.r_py, D.r_pz, {D.r_a[0], D.r_a[1], D.r_a[2]},
                     {D.r_b[0], D.r_b[1], D.r_b[2]}, D.partials, D.lm_sync, D.lm_xpub, D.pdbg,
                     D.max_in, D.max_chunks, B, D.s0};
        LmGroupCtx ctx{round, h->lm_G, D.lm_peer, D.lm_peer_flag};
        LAUNCH(FAM_LM, TRY(comm_group_launch(h->comm, &a, st, lm_group_launch, &ctx)));
      } else {
        LAUNCH(FAM_LM, k_lm_round<<<lm_padded(B) * h->lm_G, LM_THREADS, 0, st>>>(D, round, h->lm_G));
      }
    } else {
      for (int it = 0; it < 5; ++it) {  // iteration 0 + max_num_iterations = 4 candidates
        // sharded: evaluation + this rank's sums (last workgroup), then per Ceres iteration the
        // all-reduce of the 6x6 normal equations
        LAUNCH(FAM_LM, k_lm_eval<<<B * LM_EBLK, LM_THREADS, 0, st>>>(D, round, D.sharded ? 1 : 0));
        if (D.sharded) TRY(comm_allreduce(h->comm, D.lm_red, (int64_t)B * LM_NACC, LOAM_DT_F64, st));
        LAUNCH(FAM_LM, k_lm_step<<<B, 64, 0, st>>>(D, round));
      }
    }
  }
  // pose agreement across ranks before anything is stored (k_pose_adopt); the group LM round
  // (in-process ranks) leaves every rank with the same bits by construction: every rank steps on
  // the same peer slots summed in the same order
  if (D.sharded && !(multi && D.lm_peer && h->lm_G > 0)) {
    LAUNCH(FAM_OTHER, k_pose_publish<<<B, 64, 0, st>>>(D));
    if (multi)
      TRY(comm_allgather(h->comm, D.pose_x + (size_t)D.rank * B * 8, D.pose_x, (int64_t)B * 8 * sizeof(double), st));
    LAUNCH(FAM_OTHER, k_pose_adopt<<<B, 64, 0, st>>>(D));
  }
  LOAM_HIP(hipEventRecord(h->ev[2], st));
  LAUNCH(FAM_INSERT, k_insert_bucket<<<B * 2, VX_THREADS, 0, st>>>(D));
  LAUNCH(FAM_REVOX, launch_revox(h, D, st));
  LOAM_HIP(hipGetLastError());
  LOAM_HIP(hipMemcpyAsync(h->hfo[fpar].data(), D.fr, sizeof(StreamFrame) * B, hipMemcpyDeviceToHost, st));
  LOAM_HIP(hipEventRecord(h->ev_fr[fpar][1], st));
  h->spar ^= 1;  // the next frame's stacks go to the other buffers
  return LOAM_OK;
}

static int32_t mapper_replay(loam_mapper* h, const FrameRec& R, const std::vector<int>& redo);

// a queued frame is done when frame_out has written its number to the done word of its parity
// (the words only grow: a later frame of the same parity is not enqueued before this one is
// finished).  The stream is polled for errors while waiting.
static int32_t wait_word(loam_mapper* h, const unsigned long long* word, uint32_t epoch) {
  const volatile unsigned long long* w = word;
  for (uint64_t spins = 0;; ++spins) {
    if (__atomic_load_n(const_cast<const unsigned long long*>(w), __ATOMIC_ACQUIRE) >= epoch) return LOAM_OK;
    if ((spins & 1023) == 1023) {
      const hipError_t e = hipStreamQuery(h->st);
      if (e == hipSuccess) {  // the stream drained: the word must be there now
        if (__atomic_load_n(const_cast<const unsigned long long*>(w), __ATOMIC_ACQUIRE) >= epoch) return LOAM_OK;
        set_error("loam_mapper: frame finished without its done word");
        return LOAM_ERR_HIP;
      }
      if (e != hipErrorNotReady) LOAM_HIP(e);
    }
  }
}
static int32_t wait_done(loam_mapper* h, const FrameRec& R) { return wait_word(h, h->done.data() + R.fpar, R.epoch); }

// a finished frame's stream record -> the stream's stats and cube-grid centre (what
// loam_mapper_stats / _get_state report)
static void frame_stats(const StreamFrame& F, HostStream& H) {
  loam_map_stats& S = H.st;
  S.optimized = F.optimize;
  S.corner_stack = F.nc_stack;
  S.surf_stack = F.ns_stack;
  S.corner_map = F.sub_n[0];
  S.surf_map = F.sub_n[1];
  for (int r = 0; r < 2; ++r) {
    S.corner_num[r] = F.corner_num[r];
    S.surf_num[r] = F.surf_num[r];
    const LmState& L = F.lm[r];
    S.lm[r].iterations = F.optimize ? L.iteration : 0;
    S.lm[r].successful = L.successful;
    S.lm[r].invalid = L.invalid;
    S.lm[r].termination = L.term;
    S.lm[r].initial_cost = L.initial_cost;
    S.lm[r].final_cost = L.min_cost;
  }
  for (int a = 0; a < 3; ++a) {
    S.center[a] = F.center[a];
    H.cen[a] = F.cen[a];
  }
  S.valid_num = F.valid_num;
}

// the host side of one finished frame: transformUpdate (:147-151), stats, errors, timing.
// replay: a deferred frame run again for some streams (the others keep what their frame gave).
static int32_t mapper_finish_rec(loam_mapper* h, const FrameRec& R, bool replay) {
  const int B = h->B;
  float ms_total = 0, ms_opt = 0;  // (0 for a queued frame: not timed)
  if (R.chained) {
    TRY(wait_done(h, R));
  } else {
    LOAM_HIP(hipEventSynchronize(h->ev_fr[R.fpar][1]));
    LOAM_HIP(hipEventElapsedTime(&ms_total, h->ev_fr[R.fpar][0], h->ev_fr[R.fpar][1]));
    if (R.graph) ms_opt = ms_total;  // no event inside the graph (the optimisation block is most of it)
    else LOAM_HIP(hipEventElapsedTime(&ms_opt, h->ev[1], h->ev[2]));
  }
  const StreamFrame* FO = h->hfo[R.fpar].data();
  if (R.seq > h->mirror_seq) {  // the newest records the host has seen
    std::memcpy(h->hf.data(), FO, sizeof(StreamFrame) * B);
    h->mirror_seq = R.seq;
  }
  if (h->prof) {
    // the launches timed so far whose stop event has passed: this frame's, and perhaps a queued
    // frame's stack VoxelGrid (launched beside this one); the others stay listed for a later frame
    size_t kept = 0;
    for (size_t k = 0; k < h->ev_fam.size(); ++k) {
      const hipError_t q = hipEventQuery(h->ev_pool[2 * k + 1]);
      if (q == hipErrorNotReady) {
        std::swap(h->ev_pool[2 * kept], h->ev_pool[2 * k]);
        std::swap(h->ev_pool[2 * kept + 1], h->ev_pool[2 * k + 1]);
        h->ev_fam[kept++] = h->ev_fam[k];
        continue;
      }
      // a pair that cannot be timed (a launch whose enqueue failed between its events) is
      // dropped from the list, not an error of this frame
      float ms = 0;
      if (q != hipSuccess || hipEventElapsedTime(&ms, h->ev_pool[2 * k], h->ev_pool[2 * k + 1]) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      h->fam_ms[h->ev_fam[k]] += ms;
      h->fam_launches[h->ev_fam[k]]++;
    }
    h->ev_fam.resize(kept);
    // algorithmic bytes (DESIGN.md "Kernels"): what each family must read / write
    for (int s = 0; s < B; ++s) {
      const StreamFrame& F = FO[s];
      if (!F.active) continue;
      const double nst = (double)F.nc_stack + F.ns_stack;
      h->fam_bytes[FAM_STACK] += 16.0 * ((double)F.nc_in + F.ns_in + nst);
      h->fam_bytes[FAM_INSERT] += 36.0 * nst;
      if (F.optimize) {
        for (int r = 0; r < 2; ++r) {
          const double ne = F.corner_num[r], npl = F.surf_num[r], ninv = nst - ne - npl;
          const double rec = 60.0 * ne + 44.0 * npl + 4.0 * ninv;
          h->fam_bytes[FAM_CORR] += 16.0 * nst + 16.0 * (double)F.cand[r] + rec;
          h->fam_bytes[FAM_LM] += (double)F.lm[r].passes * rec;
        }
      }
    }
  }
  h->last_spar = R.fpar;
  // host bookkeeping
  int32_t status = LOAM_OK;
  std::vector<int> redo;
  for (int s = 0; s < B; ++s) {
    const StreamFrame& F = FO[s];
    HostStream& H = h->hs[s];
    if (R.active[s] && F.deferred) {  // left to the host (k_frame_prep): run again below
      redo.push_back(s);
      continue;
    }
    if (!replay || R.active[s]) H.solved_last = R.active[s] && F.active;
    if (!R.active[s] || !F.active) continue;
    H.pending = false;
    for (int i = 0; i < 7; ++i) H.pose[i] = F.pose[i];
    for (int i = 0; i < 4; ++i) H.q_wodom[i] = R.wodom[s][i];
    for (int i = 0; i < 3; ++i) H.t_wodom[i] = R.wodom[s][4 + i];
    host_transform_update(H);
    H.frame++;
    for (int m = 0; m < 2; ++m) {  // arena growth of one frame (compaction foresight)
      if (F.arena_tail[m] >= h->last_tail[s][m]) h->grow_max = std::max(h->grow_max, F.arena_tail[m] - h->last_tail[s][m]);
      h->last_tail[s][m] = F.arena_tail[m];
    }
    loam_map_stats& S = H.st;
    frame_stats(F, H);
    S.ms_total = ms_total;
    S.ms_opt = ms_opt;
    S.queued = R.chained ? 1 : 0;
    S.rerun = replay ? 1 : 0;
    if (h->prof) h->fam_bytes[FAM_REVOX] += (double)F.vx_bytes;  // counted by k_revox
    if (F.err) {
      // the frame is committed as computed (pose, insertion, re-VoxelGrid ran on the device);
      // the status says it is not trustworthy: the caller resets the stream (include/loam_core.h)
      set_error("loam_mapper_solve: stream " + std::to_string(s) + ": " + map_err_text(F.err));
      const int32_t st = (F.err & (MAP_ERR_LM_SYNC | MAP_ERR_STACK_WAIT | VH_ERR_SPIN)) ? LOAM_ERR_SYNC : LOAM_ERR_CAPACITY;
      if (status == LOAM_OK || st == LOAM_ERR_SYNC) status = st;
    }
  }
  if (!redo.empty()) {
    const int32_t rc = mapper_replay(h, R, redo);
    if (rc != LOAM_OK && (status == LOAM_OK || rc == LOAM_ERR_SYNC)) status = rc;
  }
  return status;
}

// Enqueue, on the host-prepared path, the streams `run` of a frame whose inputs and stack were
// taken earlier (R: a pending frame, or a deferred one to run again): the stack buffers of its
// parity still hold them (no stack is launched into a parity a frame in the queue holds).
static int32_t enqueue_saved(loam_mapper* h, const FrameRec& R, const std::vector<int>& run, FrameRec& out) {
  const int B = h->B;
  std::vector<HostStream> saved(h->hs.begin(), h->hs.end());  // the inputs given since
  const int spar = h->spar;
  for (int s = 0; s < B; ++s) h->hs[s].in_ready = false;
  for (int s : run) {
    HostStream& H = h->hs[s];
    H.in_ready = true;
    H.stk_launched = true;
    H.stk_seq = R.stk_seq[s];
    H.in_p[0] = R.in_p[s][0];
    H.in_p[1] = R.in_p[s][1];
    H.in_n[0] = R.in_n[s][0];
    H.in_n[1] = R.in_n[s][1];
    for (int i = 0; i < 4; ++i) H.in_q[i] = R.wodom[s][i];
    for (int i = 0; i < 3; ++i) H.in_t[i] = R.wodom[s][4 + i];
  }
  h->spar = R.fpar;
  const int32_t rc = mapper_enqueue(h, false, out);
  for (int s = 0; s < B; ++s) {  // restore the pending inputs
    HostStream& H = h->hs[s];
    const HostStream& O = saved[s];
    H.in_ready = O.in_ready;
    H.stk_launched = O.stk_launched;
    H.stk_seq = O.stk_seq;
    for (int m = 0; m < 2; ++m) {
      H.in_p[m] = O.in_p[m];
      H.in_n[m] = O.in_n[m];
    }
    for (int i = 0; i < 4; ++i) H.in_q[i] = O.in_q[i];
    for (int i = 0; i < 3; ++i) H.in_t[i] = O.in_t[i];
  }
  h->spar = spar;
  return rc;
}

// A deferred frame (k_frame_prep found a recentering or compaction due, or followed a deferred
// frame) runs again for its deferred streams on the host-prepared path, with the inputs and the
// stack it was given.  The device work queued after it, if any, left those streams alone (they
// were inactive).
static int32_t mapper_replay(loam_mapper* h, const FrameRec& R, const std::vector<int>& redo) {
  const int B = h->B;
  LOAM_HIP(hipStreamSynchronize(h->st));
  for (FrameRec& Q : h->q) {  // every frame in flight has finished on the device
    if (Q.pending) continue;
    if (Q.seq > h->mirror_seq) {  // the newest records
      std::memcpy(h->hf.data(), h->hfo[Q.fpar].data(), sizeof(StreamFrame) * B);
      h->mirror_seq = Q.seq;
    }
    // frames queued behind this one defer the same streams (k_frame_prep): no frame is queued
    // behind them until they have run again (chain_ok), so the device's deferral flags, which the
    // runs again clear, are never read meanwhile
    for (int s = 0; s < B; ++s) Q.has_deferred |= Q.active[s] && h->hfo[Q.fpar][s].deferred;
  }
  FrameRec R2;
  int32_t rc = enqueue_saved(h, R, redo, R2);
  if (rc == LOAM_OK && R2.seq) rc = mapper_finish_rec(h, R2, true);
  return rc;
}

// a pending frame at the front of the queue is enqueued (its predecessor has been waited for)
// a failed frame finished by loam_mapper_solve_async (see loam_mapper::held_rc); a hand-off
// error outranks a capacity one, the first of equal rank is kept
static void hold_status(loam_mapper* h, int32_t rc) {
  if (rc == LOAM_OK) return;
  if (h->held_rc == LOAM_OK || (rc == LOAM_ERR_SYNC && h->held_rc != LOAM_ERR_SYNC)) {
    h->held_rc = rc;
    h->held_msg = loam_last_error();
  }
}
static int32_t take_held(loam_mapper* h) {
  if (h->held_rc == LOAM_OK) return LOAM_OK;
  set_error("an earlier frame, finished by loam_mapper_solve_async, failed (" +
            std::string(h->held_rc == LOAM_ERR_SYNC ? "LOAM_ERR_SYNC" : "LOAM_ERR_CAPACITY") + "): " + h->held_msg);
  h->held_rc = LOAM_OK;
  h->held_msg.clear();
  return LOAM_ERR_EARLIER;
}

static int32_t launch_front(loam_mapper* h) {
  if (h->q.empty() || !h->q.front().pending) return LOAM_OK;
  FrameRec P = std::move(h->q.front());
  h->q.pop_front();
  std::vector<int> run;
  for (int s = 0; s < h->B; ++s)
    if (P.active[s]) run.push_back(s);
  FrameRec R;
  const int32_t rc = enqueue_saved(h, P, run, R);
  if (rc != LOAM_OK) {  // the pending frame is dropped, not run: say so
    set_error("a queued frame was dropped, not run: " + std::string(loam_last_error()));
    return rc;
  }
  R.behind = P.behind;
  if (R.seq) h->q.push_front(std::move(R));
  return LOAM_OK;
}

static int32_t finish_oldest(loam_mapper* h) {
  TRY(launch_front(h));
  if (h->q.empty()) return LOAM_OK;
  FrameRec R = std::move(h->q.front());
  h->q.pop_front();
  return mapper_finish_rec(h, R, false);
}

static int32_t settle_all(loam_mapper* h) {
  int32_t status = LOAM_OK;
  while (!h->q.empty()) {
    const int32_t rc = finish_oldest(h);
    if (rc != LOAM_OK && (status == LOAM_OK || rc == LOAM_ERR_SYNC)) status = rc;
  }
  return status;
}

// can the next frame be queued behind the one in flight?  Not when the host foresees a
// recentering for it: the initial guess from the transform known now, with a 2 m margin for the
// correction of the frame in flight.  (k_frame_prep checks exactly and defers the frame when the
// foresight was wrong.)  Compactions are queued ahead of it instead (mapper_enqueue).
static bool chain_capable(const loam_mapper* h) {
  return h->use_graph && !h->prof && !h->D.sharded && h->lm_G > 0;
}

static bool chain_ok(const loam_mapper* h) {
  if (!chain_capable(h)) return false;
  for (const FrameRec& Q : h->q)
    if (Q.has_deferred || Q.pending) return false;
  const int dims[3] = {CW, CH, CD};
  const double R = 2.0;
  for (int s = 0; s < h->B; ++s) {
    const HostStream& H = h->hs[s];
    if (!H.in_ready) continue;
    const StreamFrame& F = h->hf[s];
    double wmap[7], wodom[7], pose[7];
    for (int i = 0; i < 4; ++i) {
      wmap[i] = H.q_wmap_wodom[i];
      wodom[i] = H.in_q[i];
    }
    for (int i = 0; i < 3; ++i) {
      wmap[4 + i] = H.t_wmap_wodom[i];
      wodom[4 + i] = H.in_t[i];
    }
    pose_initial_guess(wmap, wodom, pose);
    for (int a = 0; a < 3; ++a)
      for (double d : {-R, R}) {
        const int c = cube_of(pose[4 + a] + d, F.cen[a]);
        if (c < 3 || c >= dims[a] - 3) return false;
      }
  }
  return true;
}

// Frames in the queue, oldest first, at most two: a frame in flight may have one more behind
// it, queued on the device (chained) or, when the host cannot queue it there (chain_ok), kept
// pending with its inputs and stack taken, and enqueued once its predecessor has been waited for.
// loam_mapper_wait always finishes the oldest frame, so frame f + 1 can be given before frame f
// is waited for, whichever way it runs.
static int32_t solve_async_impl(loam_mapper* h);
int32_t loam_mapper_solve_async(loam_mapper* h) {
  const int32_t rc = solve_async_impl(h);
  // a sharded rank whose HIP runtime fails here may never reach the frame's collectives: the
  // others then fail theirs at once (in-process groups) instead of waiting out the transport's
  // timeout.  (Argument, state and capacity errors are the same on every rank: identical inputs.)
  if (rc == LOAM_ERR_HIP && h && h->comm) comm_abort(h->comm);
  return rc;
}
static int32_t solve_async_impl(loam_mapper* h) {
  if (!h) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  // a third frame first finishes the oldest.  A non-OK return means the new frame was NOT
  // enqueued (a HIP / argument / state error here, or one of its own enqueue); the oldest
  // frame's own failure (a capacity or hand-off error, committed as computed) is held for the
  // next loam_mapper_wait / _solve, which return it as LOAM_ERR_EARLIER.
  if (h->q.size() >= 2) {
    const int32_t older = finish_oldest(h);
    if (older == LOAM_ERR_HIP || older == LOAM_ERR_ARG || older == LOAM_ERR_STATE) return older;
    hold_status(h, older);
  }
  TRY(launch_front(h));
  FrameRec R;
  const bool behind = !h->q.empty();
  if (h->q.empty()) {
    TRY(mapper_enqueue(h, false, R));
  } else if (chain_ok(h)) {
    TRY(mapper_enqueue(h, true, R));
  } else {  // pending: its stack now, beside the frame in flight; the rest after that frame
    TRY(launch_stacks(h));
    R.fpar = h->spar;
    R.pending = true;
    const int B = h->B;
    R.active.assign(B, 0);
    R.wodom.assign(B, std::array<double, 7>{0, 0, 0, 1, 0, 0, 0});
    R.in_p.assign(B, std::array<const float4*, 2>{nullptr, nullptr});
    R.in_n.assign(B, std::array<int, 2>{0, 0});
    R.stk_seq.assign(B, 0ull);
    bool any = false;
    for (int s = 0; s < B; ++s) {
      HostStream& H = h->hs[s];
      if (!H.in_ready) continue;
      if (!H.stk_launched) {
        set_error("loam_mapper: stack buffers of the frame's parity still in use");
        return LOAM_ERR_ARG;
      }
      any = true;
      R.active[s] = 1;
      for (int i = 0; i < 4; ++i) R.wodom[s][i] = H.in_q[i];
      for (int i = 0; i < 3; ++i) R.wodom[s][4 + i] = H.in_t[i];
      R.in_p[s] = {H.in_p[0], H.in_p[1]};
      R.in_n[s] = {H.in_n[0], H.in_n[1]};
      R.stk_seq[s] = H.stk_seq;
      H.in_ready = false;
      H.stk_launched = false;
    }
    if (!any) return LOAM_OK;
    R.seq = 1;  // (a real sequence number when it is enqueued)
    h->spar ^= 1;
  }
  R.behind = behind;
  if (R.seq) h->q.push_back(std::move(R));
  return LOAM_OK;
}

int32_t loam_mapper_wait(loam_mapper* h) {
  if (!h) return LOAM_ERR_ARG;
  if (h->q.empty()) return take_held(h);
  LOAM_HIP(hipSetDevice(h->dev));
  TRY(finish_oldest(h));  // (a pending oldest frame is enqueued first)
  // a frame waiting behind the finished one (its stack VoxelGrid already queued) is enqueued now,
  // so the device works on it while the host returns and gives the next input
  TRY(launch_front(h));
  return take_held(h);
}

int32_t loam_mapper_solve(loam_mapper* h) {
  TRY(loam_mapper_solve_async(h));
  SETTLE(h);
  return take_held(h);
}

// the newest frame's poses and stats from its early records (written after the second LM round):
// false when they cannot stand for the frame (a deferred stream, or an error flag already set),
// then the caller finishes the frame whole
static bool take_early(loam_mapper* h, FrameRec& R) {
  const StreamFrame* FE = h->hfo_early[R.fpar].data();
  for (int s = 0; s < h->B; ++s)
    if (R.active[s] && (FE[s].deferred || FE[s].err)) return false;
  for (int s = 0; s < h->B; ++s) {
    const StreamFrame& F = FE[s];
    HostStream& H = h->hs[s];
    H.solved_last = R.active[s] && F.active;
    if (!H.solved_last) continue;
    for (int i = 0; i < 7; ++i) H.pose[i] = F.pose[i];
    for (int i = 0; i < 4; ++i) H.q_wodom[i] = R.wodom[s][i];
    for (int i = 0; i < 3; ++i) H.t_wodom[i] = R.wodom[s][4 + i];
    host_transform_update(H);  // (the full finish repeats it on the same values)
    loam_map_stats& S = H.st;
    frame_stats(F, H);
    S.ms_total = 0;
    S.ms_opt = 0;
    S.queued = R.chained ? 1 : 0;
    S.rerun = 0;
  }
  R.early_seen = true;
  return true;
}

int32_t loam_mapper_solve_pose(loam_mapper* h) {
  if (!h) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  if (!h->early) {  // the frames' sequences gain the early records: recapture the graphs
    SETTLE(h);
    for (auto& gp : h->gexec)
      for (auto& g : gp)
        if (g) {
          (void)hipGraphExecDestroy(g);
          g = nullptr;
        }
    h->early = true;
  }
  TRY(loam_mapper_solve_async(h));  // queued behind the previous frame, as the pipelined solves
  while (h->q.size() > 1) {  // the previous frame: its insertion and re-VoxelGrid ran meanwhile
    const int32_t older = finish_oldest(h);
    if (older == LOAM_ERR_HIP || older == LOAM_ERR_ARG || older == LOAM_ERR_STATE) return older;
    hold_status(h, older);
  }
  TRY(launch_front(h));  // (a frame kept pending behind it is enqueued now)
  if (h->q.empty()) return take_held(h);
  FrameRec& R = h->q.front();
  bool early = R.graph && !R.pending;
  if (early) TRY(wait_word(h, h->done_early.data() + R.fpar, R.epoch));
  if (!early || !take_early(h, R)) {  // the frame whole: its status now
    const int32_t rc = finish_oldest(h);
    if (rc != LOAM_OK) return rc;
  }
  return take_held(h);
}

int32_t loam_mapper_debug_counters(loam_mapper* h, uint64_t* out, int32_t n, int32_t reset) {
  SETTLE(h);
  if (!h || !out || n < 0 || n > LOAM_DEBUG_COUNTERS) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  LOAM_HIP(hipStreamSynchronize(h->st));
  LOAM_HIP(hipMemcpy(out, h->D.dbg, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
  if (reset) LOAM_HIP(hipMemset(h->D.dbg, 0, sizeof(uint64_t) * LOAM_DEBUG_COUNTERS));
  return LOAM_OK;
}

int32_t loam_mapper_set_profiling(loam_mapper* h, int32_t enable) {
  SETTLE(h);
  if (!h) return LOAM_ERR_ARG;
  h->prof = enable != 0;
  h->ev_fam.clear();  // (settled: every timed launch has been read)
  return LOAM_OK;
}

int32_t loam_mapper_kernel_times(loam_mapper* h, loam_kernel_times* out) {
  SETTLE(h);
  if (!h || !out) return LOAM_ERR_ARG;
  for (int f = 0; f < LOAM_KFAM_COUNT; ++f) {
    out->ms[f] = f < NFAM ? h->fam_ms[f] : 0.0;
    out->launches[f] = f < NFAM ? h->fam_launches[f] : 0;
    out->bytes[f] = f < NFAM ? h->fam_bytes[f] : 0.0;
  }
  return LOAM_OK;
}

int32_t loam_mapper_reset_kernel_times(loam_mapper* h) {
  SETTLE(h);
  if (!h) return LOAM_ERR_ARG;
  for (int f = 0; f < NFAM; ++f) {
    h->fam_ms[f] = h->fam_bytes[f] = 0.0;
    h->fam_launches[f] = 0;
  }
  return LOAM_OK;
}

int32_t loam_mapper_pose(loam_mapper* h, int32_t s, double* q_w, double* t_w) {
  SETTLE_RESULTS(h);
  TRY(check_stream(h, s));
  if (!q_w || !t_w) return LOAM_ERR_ARG;
  const HostStream& H = h->hs[s];
  if (H.skip) {
    for (int i = 0; i < 4; ++i) q_w[i] = H.q_hf[i];
    for (int i = 0; i < 3; ++i) t_w[i] = H.t_hf[i];
  } else {
    for (int i = 0; i < 4; ++i) q_w[i] = H.pose[i];
    for (int i = 0; i < 3; ++i) t_w[i] = H.pose[4 + i];
  }
  return LOAM_OK;
}

int32_t loam_mapper_stats(loam_mapper* h, int32_t s, loam_map_stats* st) {
  SETTLE_RESULTS(h);
  TRY(check_stream(h, s));
  if (!st) return LOAM_ERR_ARG;
  *st = h->hs[s].st;
  return LOAM_OK;
}

int32_t loam_mapper_get_state(loam_mapper* h, int32_t s, int32_t* cen, double* q, double* t) {
  SETTLE_RESULTS(h);
  TRY(check_stream(h, s));
  if (!cen || !q || !t) return LOAM_ERR_ARG;
  for (int a = 0; a < 3; ++a) cen[a] = h->hs[s].cen[a];
  for (int i = 0; i < 4; ++i) q[i] = h->hs[s].q_wmap_wodom[i];
  for (int i = 0; i < 3; ++i) t[i] = h->hs[s].t_wmap_wodom[i];
  return LOAM_OK;
}

// cell index of cubes [c0, c1) of (stream, map) after host-side changes
static int32_t build_cube_index(loam_mapper* h, int32_t s, int32_t m, int32_t c0, int32_t c1) {
  LOAM_HIP(hipSetDevice(h->dev));
  // the device copy of the stream record supplies arena_active: refresh it first
  LOAM_HIP(hipMemcpyAsync(h->D.fr + s, &h->hf[s], sizeof(StreamFrame), hipMemcpyHostToDevice, h->st));
  MapperDev D = h->D;
  D.cube_tab = h->cube_tab[h->parity];
  const int3 cen = make_int3(h->hf[s].cen[0], h->hf[s].cen[1], h->hf[s].cen[2]);
  k_cube_index<<<c1 - c0, VX_THREADS, 0, h->st>>>(D, s, m, c0, c1, cen);
  LOAM_HIP(hipGetLastError());
  LOAM_HIP(hipStreamSynchronize(h->st));
  return LOAM_OK;
}

int32_t loam_mapper_set_state(loam_mapper* h, int32_t s, const int32_t* cen, const double* q, const double* t) {
  SETTLE(h);
  TRY(check_stream(h, s));
  if (!cen || !q || !t) return LOAM_ERR_ARG;
  bool moved = false;
  for (int a = 0; a < 3; ++a) {
    moved |= h->hf[s].cen[a] != cen[a];
    h->hf[s].cen[a] = h->hs[s].cen[a] = cen[a];
  }
  for (int i = 0; i < 4; ++i) h->hs[s].q_wmap_wodom[i] = h->hf[s].wmap[i] = q[i];
  for (int i = 0; i < 3; ++i) h->hs[s].t_wmap_wodom[i] = h->hf[s].wmap[4 + i] = t[i];
  if (moved)  // cube world positions changed: rebuild every cube's cell index
    for (int m = 0; m < 2; ++m) TRY(build_cube_index(h, s, m, 0, NCUBE));
  return LOAM_OK;
}

int32_t loam_mapper_cube_count(loam_mapper* h, int32_t s, int32_t which, int32_t cube) {
  SETTLE(h);
  TRY(check_stream(h, s));
  if (which < 0 || which > 1 || cube < 0 || cube >= NCUBE) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  uint2 v;
  LOAM_HIP(hipMemcpy(&v, h->cube_tab[h->parity] + ((size_t)s * 2 + which) * NCUBE + cube, sizeof(uint2), hipMemcpyDeviceToHost));
  return (int32_t)v.y;
}

int32_t loam_mapper_cube_copy(loam_mapper* h, int32_t s, int32_t which, int32_t cube, float* out) {
  SETTLE(h);
  TRY(check_stream(h, s));
  if (which < 0 || which > 1 || cube < 0 || cube >= NCUBE || !out) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  uint2 v;
  LOAM_HIP(hipMemcpy(&v, h->cube_tab[h->parity] + ((size_t)s * 2 + which) * NCUBE + cube, sizeof(uint2), hipMemcpyDeviceToHost));
  const float4* base = h->D.arena + (((size_t)s * 2 + which) * 2 + h->hf[s].arena_active[which]) * (size_t)h->D.map_cap;
  if (v.y) LOAM_HIP(hipMemcpy(out, base + v.x, sizeof(float4) * v.y, hipMemcpyDeviceToHost));
  return (int32_t)v.y;
}

int32_t loam_mapper_stack_copy(loam_mapper* h, int32_t s, int32_t which, float* out, int32_t cap) {
  SETTLE(h);
  TRY(check_stream(h, s));
  if (which < 0 || which > 1 || (cap > 0 && !out)) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  const int32_t n = which == 0 ? h->hf[s].nc_stack : h->hf[s].ns_stack;
  if (n > cap) return n;  // the count only
  if (n) {
    LOAM_HIP(hipMemcpy(out, h->stack_buf[h->last_spar][which] + (size_t)s * h->D.max_in, sizeof(float4) * n,
                       hipMemcpyDeviceToHost));
  }
  return n;
}

int32_t loam_mapper_cube_set(loam_mapper* h, int32_t s, int32_t which, int32_t cube, const float* pts, int32_t n) {
  SETTLE(h);
  TRY(check_stream(h, s));
  if (which < 0 || which > 1 || cube < 0 || cube >= NCUBE || n < 0 || (n > 0 && !pts)) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  std::vector<float> mine;
  if (h->D.sharded) {  // a sharded handle stores the points of the blocks its rank owns
    for (int i = 0; i < n; ++i)
      if (loam_shard_owner(pts + 4 * (size_t)i, h->D.leaf[which], h->D.nrank) == h->D.rank) mine.insert(mine.end(), pts + 4 * (size_t)i, pts + 4 * (size_t)i + 4);
    pts = mine.data();
    n = (int32_t)(mine.size() / 4);
  }
  StreamFrame& F = h->hf[s];
  uint32_t& tail = F.arena_tail[which];
  if (tail + (uint32_t)n > (uint32_t)h->D.map_cap) {
    set_error("loam_mapper_cube_set: arena full");
    return LOAM_ERR_CAPACITY;
  }
  float4* base = h->D.arena + (((size_t)s * 2 + which) * 2 + F.arena_active[which]) * (size_t)h->D.map_cap;
  if (n) LOAM_HIP(hipMemcpy(base + tail, pts, sizeof(float4) * n, hipMemcpyHostToDevice));
  uint2 v = make_uint2(tail, (uint32_t)n);
  tail += n;
  LOAM_HIP(hipMemcpy(h->cube_tab[h->parity] + ((size_t)s * 2 + which) * NCUBE + cube, &v, sizeof(uint2), hipMemcpyHostToDevice));
  const uint32_t zero = 0;  // caller content: not known to be a VoxelGrid fixed point
  LOAM_HIP(hipMemcpy(h->D.stable_tok + ((size_t)s * 2 + which) * NCUBE + cube, &zero, sizeof(zero), hipMemcpyHostToDevice));
  return build_cube_index(h, s, which, cube, cube + 1);
}

static int32_t pub_reserve(loam_mapper* h, size_t n) {
  if (n <= h->pub_cap) return LOAM_OK;
  if (h->d_pub) (void)hipFree(h->d_pub);
  h->d_pub = nullptr;
  h->pub_cap = 0;
  LOAM_HIP(hipMalloc(&h->d_pub, sizeof(float4) * std::max<size_t>(n, 1)));
  h->pub_cap = n;
  return LOAM_OK;
}

int32_t loam_mapper_map_copy(loam_mapper* h, int32_t s, float* out, int64_t cap) {
  SETTLE(h);
  TRY(check_stream(h, s));
  if (cap < 0 || (cap > 0 && !out)) return LOAM_ERR_ARG;
  LOAM_HIP(hipSetDevice(h->dev));
  MapperDev D = h->D;
  D.cube_tab = h->cube_tab[h->parity];
  // the device stream record supplies arena_active (current after every solve / set)
  LOAM_HIP(hipMemcpyAsync(h->D.fr + s, &h->hf[s], sizeof(StreamFrame), hipMemcpyHostToDevice, h->st));
  k_map_scan<<<1, VX_THREADS, 0, h->st>>>(D, s, h->d_map_off);
  uint32_t total = 0;
  LOAM_HIP(hipMemcpyAsync(&total, h->d_map_off + 2 * NCUBE, sizeof(uint32_t), hipMemcpyDeviceToHost, h->st));
  LOAM_HIP(hipStreamSynchronize(h->st));
  if ((int64_t)total > cap) return (int32_t)total;  // the count only
  if (total) {
    TRY(pub_reserve(h, total));
    k_map_gather<<<512, 256, 0, h->st>>>(D, s, h->d_map_off, h->d_pub);
    LOAM_HIP(hipGetLastError());
    LOAM_HIP(hipMemcpyAsync(out, h->d_pub, sizeof(float4) * total, hipMemcpyDeviceToHost, h->st));
    LOAM_HIP(hipStreamSynchronize(h->st));
  }
  return (int32_t)total;
}

static int32_t register_common(loam_mapper* h, int32_t s, const float* in, int32_t n, float* out, bool device) {
  TRY(check_stream(h, s));
  if (n < 0 || (n > 0 && (!in || !out))) return LOAM_ERR_ARG;
  if (n == 0) return 0;
  LOAM_HIP(hipSetDevice(h->dev));
  MapPose P;
  TRY(loam_mapper_pose(h, s, P.x, P.x + 4));
  const float4* src = reinterpret_cast<const float4*>(in);
  float4* dst = reinterpret_cast<float4*>(out);
  if (!device) {
    TRY(pub_reserve(h, n));
    LOAM_HIP(hipMemcpyAsync(h->d_pub, in, sizeof(float4) * n, hipMemcpyHostToDevice, h->st));
    src = dst = h->d_pub;
  }
  k_register<<<std::min(1024, (n + 255) / 256), 256, 0, h->st>>>(src, dst, n, P);
  LOAM_HIP(hipGetLastError());
  if (!device) LOAM_HIP(hipMemcpyAsync(out, h->d_pub, sizeof(float4) * n, hipMemcpyDeviceToHost, h->st));
  LOAM_HIP(hipStreamSynchronize(h->st));
  return n;
}

int32_t loam_mapper_register_cloud(loam_mapper* h, int32_t s, const float* in, int32_t n, float* out) {
  SETTLE(h);
  return register_common(h, s, in, n, out, false);
}

int32_t loam_mapper_register_cloud_device(loam_mapper* h, int32_t s, const float* d_in, int32_t n, float* d_out) {
  SETTLE(h);
  return register_common(h, s, d_in, n, d_out, true);
}

}  // extern "C"

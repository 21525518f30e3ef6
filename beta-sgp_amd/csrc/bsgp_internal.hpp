// bsgp_internal.hpp — structures shared by the kernels (bsgp_solver.hip) and
// the C-ABI host layer (bsgp_api.hip).  Not part of the public interface.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/bsgp.h"
#include "bsgp_device.hpp"

namespace bsgp {

// Per-image solver state carried between the phase kernels (device memory).
struct ImgState {
  int par, Xones, stop, iter, epoch;
  int bar_base;  // team barriers completed before the next kernel (T > 1)
  int64_t E_p, E_ls, ls_passes, status, ls_series;
  int64_t proj_passes, proj_list;  // projection passes over the image / list entries read
  double sc, flux, bks_scalar, lo, hi, Dcoeff, tol, t0;
  double fv, alpha, tau, lr, init_lr, beta, lam_p, gd, lam;
  // projection history for the first pass's split bracket (cached_projection):
  // the last multiplier over the step length it was found at, and the last
  // search's first secant point over its root (0: none yet)
  double lam_ratio, kappa;
  double konst;  // lambda-independent objective sum at `beta` (sum s*gn^b / sum gn)
  // compact observed image (params.gn_compact): 0 = gn_s stored in f64; 1 = the
  // raw counts stored in f32, gn_s = raw (scale_data 0/2); 2 = gn_s = raw / sc.
  // gfill is the null-pixel value vmin*eps^2 (sgp.py:202-204).
  int g32;
  double gfill;
  double Valpha[32];
  double Fold[32];
};

// Everything a phase kernel needs (passed by value: kernel-argument loads are
// scalar, so plan geometry and pointers stay in SGPRs).
// Column passes run inside the phase kernels for one-workgroup images
// instead of as k_col launches: A's at the end of k_dir (bit 0) or at the
// start of k_ls (bit 2), AT's at the end of k_ls (bit 1).  Measured on C3
// (A/B): AT's in k_ls +4.5 %; A's in k_dir -25 % (252 VGPRs + scratch: the
// projection state stays live), A's also in k_ls -1 % (spills at 168 VGPRs).
#ifndef BSGP_FUSE_COL
#define BSGP_FUSE_COL 2
#endif
// teams of per-wave plans (C2): which column passes their row kernels run
// after a team barrier instead of a k_col launch
#ifndef BSGP_FUSE_COL_TEAM
#define BSGP_FUSE_COL_TEAM 0
#endif
// fused-column code compiled into the kernels (a pass not compiled in costs no
// registers in the kernels that never run it)
#define BSGP_FUSE_COL_CODE (BSGP_FUSE_COL | BSGP_FUSE_COL_TEAM)
// teams keep their projection lists in LDS when they fit (0: global, A/B)
#ifndef BSGP_LIST_LDS
#define BSGP_LIST_LDS 1
#endif

// numpy float32 reduction program of a plan's N (bsgp_api.hip pairwise_program):
// [nleaf][2] leaves (start, len), [nnode][2] node operands (value indices),
// [nlev + 1] level offsets into the nodes, [nchunk] root value of each chunk.
struct PwProg {
  const int* prog;
  int nleaf, nnode, nlev, nchunk;
};

struct SolveArgs {
  Geo g;
  bsgp_params prm;
  bsgp_inputs in;
  bsgp_outputs out;
  int B;
  int img0, nimg;      // this launch's sub-batch [img0, img0 + nimg)
  ImgState* st;        // [B]
  int* active;         // images not yet stopped: B at the start (the host sets it); the setup
                       // and k_bb count each stopping image down
  int* done_host;      // host-mapped word: the solve's `seq` once `active` reaches 0 (the
                       // host's lookahead polling of data-dependent stop rules), or nullptr
  int seq;             // this solve's sequence number (done_host)
  double* ws;          // per-image slots
  size_t slot_stride;  // doubles per slot
  size_t vec_stride;   // doubles per image vector (N rounded up to 32)
  size_t lds_fft_bytes;
  // teams (T workgroups per image; T = 1: one workgroup, none of these used)
  int T;
  int Tc;               // workgroups per image of k_col (no reductions there: not a team)
  int fuse_col;         // T == 1: BSGP_FUSE_COL (which phase kernels run the column passes)
  double* tpart;        // [B][kPartBufs][T][kMaxRed] reduction partials
  unsigned int* tctr;   // [B][kTeamWords] barrier words, then the timeout word; zeroed per solve
  int* tfail;           // set by a timed-out barrier spin
  // projection pixel lists (proj_cache): per image two arrays (y, X) of
  // lcap * T * kBlock doubles; entry k of global thread gt at k*T*kBlock + gt
  double* plist;
  size_t plist_stride;  // doubles per image (both arrays)
  int lcap;             // list capacity per thread (pixels one thread streams)
  int list_lds;         // teams: list entries per thread kept in the transform buffers' LDS
  PwProg pw;            // numpy float32 sum order over N (params.gn_f32)
  int storage;          // BSGP_STORAGE_F64 / F32 (iteration vectors, Bufs<V>)
  size_t spec_off;      // doubles from a slot's start to its spectrum
  int ls_cap;           // line-search trial cap: lam = beta^(k-1) < 1e-12 ends the search
                        // (sgp.py:336) by trial ceil(log 1e-12 / log beta) + 1 for 0 < beta < 1
  unsigned spin_limit;  // persistent solver: s_sleep polls before a hand-off wait gives up
                        // (status bit 4); 2^26 unless BSGP_SPIN_LIMIT says otherwise (tests)
  int fold_setup;       // persistent solver, slot order: every image's setup is the first
                        // task of its chain inside k_persist (no k_setup launch)
};

hipError_t launch_setup(const SolveArgs& a, size_t lds, hipStream_t s);
// ev: NULL, or 6 events recorded around the kernels of one iteration (profiled solves)
hipError_t launch_iteration(const SolveArgs& a, int K, size_t lds, hipStream_t s,
                            hipEvent_t* ev = nullptr);
hipError_t launch_track(const SolveArgs& a, int it, hipStream_t s);
hipError_t launch_build_tf(const Geo& g, const double* kc, cd* spec, cd* tf, double scale,
                           int conj, size_t lds, hipStream_t s);
hipError_t launch_build_tfs(const Geo& g, int n, const double* kc, size_t kc_stride, cd* spec,
                            size_t spec_stride, cd* tf, size_t tf_stride, double scale, int conj,
                            size_t lds, hipStream_t s);
hipError_t launch_place_psfs(const Geo& g, int n, const double* psfs, int kh, int kw, int circ,
                             double* kc, double* sums, hipStream_t s);
hipError_t launch_apply_op(const Geo& g, int B, int transpose, const double* x, double* out,
                           cd* specws, size_t spec_stride, int grid, size_t lds, hipStream_t s);
hipError_t launch_apply_op_split(const Geo& g, int B, int transpose, const double* x,
                                 double* out, cd* specws, size_t spec_stride, int per, size_t lds,
                                 hipStream_t s);
hipError_t launch_project_df(int n, double b, const double* c, const double* dia, ProjClip clip,
                             double lam0, double dlam0, double tol_lam, int biter, int siter,
                             int max_projs, double* x, double* info, hipStream_t s);
hipError_t launch_beta_div(int n, const double* y, const double* x, double beta, double* out,
                           hipStream_t s);
hipError_t launch_beta_div_deriv(int64_t n, const double* y, const double* x, double beta,
                                 double* out, hipStream_t s);
hipError_t launch_grad_parts(int64_t n, const double* den, const double* gn, double beta,
                             double* pow1, double* w, hipStream_t s);
hipError_t set_solver_lds_limit(size_t bytes);
// workgroups of every team kernel of a build (coop, storage) one CU holds at once
hipError_t team_resident_per_cu(bool coop, int storage, size_t lds, int* per_cu);
hipError_t launch_extract_tiles(const double* img, int W, const int* boxes, int n, int th, int tw,
                                double* out, hipStream_t s);
hipError_t launch_coadd_tiles(const double* tiles, int n, int th, int tw, const int* boxes, int H,
                              int W, double* mean, double* footprint, hipStream_t s);
hipError_t launch_fits_to_f64(const void* raw, int64_t n, int bitpix, double bscale, double bzero,
                              double* out, hipStream_t s);
struct PsfModel;
hipError_t launch_psf_stamps(const PsfModel& m, const double* xy, int n, int spatial,
                             int normalize, double* out, hipStream_t s);
hipError_t phase_prof(unsigned long long* out, int n, int reset);
// persistent task-queue solver (bsgp_persist.hip): one launch runs every
// iteration of every image; queue = dequeue counter, done[B] = iterations
// published per image (both zeroed per solve)
hipError_t launch_persist(const SolveArgs& a, int K, size_t lds, hipStream_t s, unsigned* queue,
                          unsigned* done, int grid);
hipError_t persist_resident_per_cu(const SolveArgs& a, int K, size_t lds, int* per_cu);
hipError_t persist_phase_prof(unsigned long long* out, int n, int reset);
void persist_kernels_all(std::vector<const void*>& f);

// Cooperative plans (Geo::coop) run the phase kernels of bsgp_solver_c512.hip:
// the same kernels with 512-thread workgroups (two waves per SIMD per
// workgroup where a long transform's LDS allows one or two workgroups per CU).
// cooperative plans: at most this many thread groups per workgroup run
// transforms side by side (bsgp_device.hpp coop passes), and the column
// kernel's groups (0: the same as the other kernels)
// plans whose per-wave transforms fit the LDS at three workgroups per CU (but
// not four) take them instead of the cooperative build when this is <= 3
// (runtime override: BSGP_PERWAVE_MIN_WG)
#ifndef BSGP_PERWAVE_MIN_WG
#define BSGP_PERWAVE_MIN_WG 2  // per-wave over cooperative (A/B): 375^2 tiles at 3 WG/CU, 1024 per
                               // launch, 68.6 k -> 87.5 k image-it/s; 450^2 at 2 WG/CU 48.3 -> 59.7 k
#endif
#ifndef BSGP_PERWAVE_TW
#define BSGP_PERWAVE_TW 1
#endif
#ifndef BSGP_COOP_GROUPS
#define BSGP_COOP_GROUPS 4
#endif
#ifndef BSGP_POLL_LOOKAHEAD
#define BSGP_POLL_LOOKAHEAD 1  // data-dependent stop rules: lookahead polling (bsgp_api.hip)
#endif
#ifndef BSGP_COOP_TW2
#define BSGP_COOP_TW2 1  // two-level LDS twiddles for cooperative 2048-point transforms
#endif
#ifndef BSGP_SPEC_PAD
#define BSGP_SPEC_PAD 0  // rows of padding per stored spectrum column (even)
#endif
#ifndef BSGP_VEC_PAD
#define BSGP_VEC_PAD 0  // elements of padding after every per-image slot vector (multiple of 32)
#endif
#ifndef BSGP_COOP_ELEMS
#define BSGP_COOP_ELEMS 8  // elements per thread a group may take when one batch leaves one group
#endif
#ifndef BSGP_COOP_COLGROUPS
#define BSGP_COOP_COLGROUPS 0  // 375^2 tiles: k_col on 4 groups 1.49 -> 0.68 ms (A/B)
#endif
#ifndef BSGP_COOP512
#define BSGP_COOP512 1
#endif
constexpr int kCoopBlock = BSGP_COOP512 ? 512 : kBlock;
// threads per workgroup of a plan's phase kernels
__host__ __device__ inline int plan_block(const Geo& g) { return g.coop ? kCoopBlock : kBlock; }
// plans whose persistent solve runs the application-size build (bsgp_persist_app.hip):
// per-wave, float64 storage, a 400- or 480-point row or column transform
inline bool app_static_plan(const Geo& g, int storage) {
  const bool app_n = g.fp.n == 400 || g.fp.n == 480 || g.fq.n == 400 || g.fq.n == 480;
  return !g.coop && storage == BSGP_STORAGE_F64 && app_n;
}

}  // namespace bsgp

// bsgp_solver_c512.hip (C linkage: its types live in namespace bsgp_c512; the
// argument block is this header's SolveArgs, same layout)
extern "C" {
size_t bsgp_c512_args_size(void);
int bsgp_c512_block(void);
int bsgp_c512_waves(void);
hipError_t bsgp_c512_launch_setup(const void* a, size_t lds, hipStream_t s);
hipError_t bsgp_c512_launch_iteration(const void* a, int K, size_t lds, hipStream_t s,
                                      hipEvent_t* ev);
hipError_t bsgp_c512_team_resident(int storage, size_t lds, int* per_cu);
hipError_t bsgp_c512_set_lds_limit(size_t bytes);
// the cooperative plans' persistent solver (bsgp_persist_c512.hip)
hipError_t bsgp_c512_launch_persist(const void* a, int K, size_t lds, hipStream_t s,
                                    unsigned* queue, unsigned* done, int grid);
hipError_t bsgp_c512_persist_resident(const void* a, int K, size_t lds, int* per_cu);
hipError_t bsgp_c512_persist_set_lds_limit(size_t bytes);
// the application-size persistent build (bsgp_persist_app.hip): per-wave plans
// of float64 storage whose row or column transform has 400 or 480 points
size_t bsgp_app_args_size(void);
hipError_t bsgp_app_launch_persist(const void* a, int K, size_t lds, hipStream_t s,
                                   unsigned* queue, unsigned* done, int grid);
hipError_t bsgp_app_persist_resident(const void* a, int K, size_t lds, int* per_cu);
hipError_t bsgp_app_persist_set_lds_limit(size_t bytes);
hipError_t bsgp_app_phase_prof(unsigned long long* out, int n, int reset);
hipError_t bsgp_c512_phase_prof(unsigned long long* out, int n, int reset);
}

/* bsgp.h — C ABI of the MI355X beta-SGP engine (libbsgp.so, gfx950).
 *
 * The reference boundary is a Python API, not an FFI: restoration/sgp.py's
 * sgp() (sgp.py:41-47), sgp_betaDiv() (sgp.py:506-513), the betaDiv family
 * (sgp.py:441-503) and flux_conserve_proj.projectDF() (flux_conserve_proj.py:7).
 * The drop-in Python modules beta-sgp_amd/sgp.py and
 * beta-sgp_amd/flux_conserve_proj.py keep those signatures and bind the entry
 * points below through ctypes (INTEGRATION.md shows the stubs).
 *
 * Conventions
 *  - plain C types only; device pointers are HBM buffers of the calling
 *    process's current HIP device; `stream` is a hipStream_t passed as void*
 *    (NULL = the null stream). Entry points are asynchronous on `stream`
 *    unless their comment says otherwise.
 *  - every function returns BSGP_OK (0) or a negative status; the message of
 *    the last failure on the calling thread is in bsgp_last_error().
 *  - all arrays are C-contiguous little-endian float64; an image batch is
 *    [B][H][W].
 *  - a plan is not thread-safe: one plan per device per host thread.
 */
#ifndef BSGP_H_
#define BSGP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BSGP_OK 0
#define BSGP_ERR_ARG (-1)          /* bad argument / shape                       */
#define BSGP_ERR_HIP (-2)          /* a HIP runtime call failed                  */
#define BSGP_ERR_UNSUPPORTED (-3)  /* geometry the kernels do not cover (yet)    */
#define BSGP_ERR_PSF (-4)          /* PSF not normalised (sgp.py:97-102)         */

/* conv_mode: which A/AT the solver uses.
 *  BSGP_CONV_CIRCULAR    use_original_SGP_Afunction=True  (sgp.py:108-120):
 *                        A(x)=Re ifft2(fft2(fftshift(psf)) . fft2(x)), AT uses conj;
 *                        psf must have the image's shape.
 *  BSGP_CONV_LINEAR_FILL use_original_SGP_Afunction=False (sgp.py:121-161):
 *                        astropy convolve_fft(x, psf/sum(psf)) with zero fill,
 *                        cropped; AT convolves with psf.T. */
#define BSGP_CONV_CIRCULAR 0
#define BSGP_CONV_LINEAR_FILL 1

#define BSGP_VARIANT_KL 0   /* sgp()          sgp.py:41-438  */
#define BSGP_VARIANT_BETA 1 /* sgp_betaDiv()  sgp.py:506-895 */

typedef struct bsgp_plan_s* bsgp_plan;

/* Every keyword argument of sgp()/sgp_betaDiv() that reaches the iteration.
 * Field meanings are the reference's (sgp.py:48-77, 515-542). */
typedef struct {
  int32_t variant;        /* BSGP_VARIANT_*                                        */
  int32_t init_recon;     /* 0 zeros, 1 x0 given (randn, sgp.py:169-170), 2 gn, 3 flat */
  int32_t proj_type;      /* 0 clamp at 0, 1 flux-conserving projectDF             */
  int32_t stop_criterion; /* 0/1 MAXIT only, 2 step norm, 3 rel. decrease, 4 discrepancy */
  int32_t MAXIT;
  int32_t M_alpha;        /* <= 32 */
  int32_t M;              /* <= 32 */
  int32_t max_projs;
  double gamma, beta, alpha, alpha_min, alpha_max, tau;
  double ccd_sat_level;   /* used when has_sat */
  double betaParam, lr, lr_exp_param;
  double tol_convergence;
  double prescaled_scaling; /* scale_data == 2: the scaling the caller applied    */
  double prescaled_tol4;    /* scale_data == 2 and stop_criterion 4: 1+1/mean(gn) */
  int32_t has_sat;
  int32_t scale_data;     /* 0 none, 1 scaling = max(gn) on device (sgp.py:193-199),
                             2 inputs already scaled by the caller in their own dtype:
                             gn, bkg, x0 are used as given (x0 required); with
                             gn_f32, 0 and 1 run the float32 prelude on the device
                             (see below)                                           */
  int32_t verbose;        /* only changes tol**2 for stop_criterion 2 (sgp.py:291-294) */
  int32_t adapt_beta;
  int32_t schedule_lr;
  int32_t bkg_is_map;     /* bkg is [B][H][W] instead of [B] scalars               */
  int32_t ls_spec;        /* line-search lambdas evaluated per pass (1..8); 1 when adapt_beta */
  int32_t ls_series;      /* 1: small trial steps from the moment series (general beta) */
  int32_t streams;        /* sub-batches run on this many streams (1..16: the caller's + 15 plan
                             streams) so phases overlap; more than GPU_MAX_HW_QUEUES share queues */
  int32_t team;           /* workgroups cooperating on one image: 0 = auto (spread the
                             batch over the CUs when B is small), 1 = one per image,
                             k > 1 = at most k (capped so every workgroup is resident) */
  int32_t proj_cache;     /* 1: projectDF evaluations whose multiplier falls inside a
                             bracket known to hold the root read only the pixels that
                             change state inside it (a per-lane list written by the
                             last full pass); 0: every evaluation streams the image */
  int32_t gn_compact;     /* 1: an image whose observed values are all finite and exact
                             in f32 (counts, or f32 FITS data) keeps them in f32 and
                             recomputes the scaled gn/scaling (and the null-pixel fill)
                             on every read, bit-identical to f64 storage; the line
                             search reads half the bytes of gn. 0: f64 storage */
  int32_t gn_f32;         /* 1: gn is the reference's float32 image (scale_data == 2: the
                             caller scaled it in float32).  Under numpy 1.x promotion the
                             beta objective then sums s*gn**beta as float32 terms
                             (exponent rounded to float32) with numpy's float32 pairwise
                             reduction, and rounds (s*beta)*gn to float32 before the
                             multiply by den**(beta-1) (sgp.py:457-458); the device
                             reproduces both.  With proj_type 0 the first iteration's
                             scaling matrix clips to float32 bounds (sgp.py:726-729). */
  int32_t beta0_general;  /* 1: every in->beta0[b] is neither 0 nor 1, so a batch with
                             per-image betas can use the general-beta kernels */
  int32_t flux_f32;       /* gn_f32 with scale_data 0/1: in->flux holds numpy float32
                             values, divided by the scaling in float32 (sgp.py:666) */
  int32_t persistent;     /* 1: one-workgroup images (team 1, per-wave transforms, no
                             err / x_iter) run every iteration in ONE persistent launch
                             that dequeues (iteration, image) tasks; the same device
                             code per iteration, bit-identical results.  0: one launch
                             per phase and iteration on sub-batch streams */
} bsgp_params;
/* gn_f32 with scale_data 0 or 1 (ABI 3): the float32 prelude of sgp.py:620-666
 * runs on the device.  in->gn holds the raw float32 image values (exact in
 * float64), in->bkg float64 backgrounds, in->flux the raw provided flux; the
 * device takes scaling = max(gn), gn/scaling and (init_recon 2) x/scaling in
 * float32, the null-pixel fill rounded to float32, stop rule 4's 1 + 1/mean(gn)
 * from numpy's float32 mean, and init_recon 3's flat start rounded to float32,
 * as numpy 1.x evaluates them for a float32 image (bkg/scaling, a float64
 * flux/scaling and x0/scaling stay float64).  Not covered (the caller scales):
 * float32 backgrounds, and init_recon 3 without a flux and with a scalar bkg
 * (numpy sums that start in float32). */

/* Storage of the per-image iteration vectors (bsgp_plan_create). */
#define BSGP_STORAGE_F64 0
#define BSGP_STORAGE_F32 1

/* Device inputs of a batched solve. */
typedef struct {
  const double* gn;    /* [B][H][W] observed images (any scale; scaled on device) */
  const double* bkg;   /* [B] or [B][H][W] (bkg_is_map)                           */
  const double* flux;  /* [B] precomputed flux or NULL = sum(gn - bkg); unscaled, or
                          already scaled when scale_data == 2 (sgp.py:208-211)      */
  const double* x0;    /* [B][H][W] initial x (init_recon == 1, or scale_data == 2), else NULL */
  const double* beta0; /* [B] per-image initial betaParam or NULL = params.betaParam */
  const double* obj;   /* [B][H][W] ground truth (unscaled) for out->err, or NULL  */
} bsgp_inputs;

/* Device outputs of a batched solve.  MAXIT1 = MAXIT + 1. */
typedef struct {
  double* x;           /* [B][H][W] restored image (x * scaling)                  */
  int32_t* iters;      /* [B] iterations (the reference's returned iter_)         */
  double* discr;       /* [B][MAXIT1] discrepancy 2/N*scaling*f (sgp.py:276,392)  */
  double* times;       /* [B][MAXIT1] seconds since solve start (sgp.py:391), may be NULL */
  double* crit;        /* [B][MAXIT1] stop-rule value per iteration, may be NULL  */
  int32_t* flags;      /* [B][MAXIT1] bit0: fv >= fr warning (sgp.py:351, 803);
                          bits 8..23: line-search trials of iteration k (the
                          betaDiv calls of sgp.py:782 / objective evaluations of
                          :334 in iteration k); may be NULL */
  double* beta_final;  /* [B] final betaParam (sgp.py:892), may be NULL           */
  int64_t* counters;   /* [B][8]: proj evals E_p, line-search trials E_ls,
                          line-search passes over the image, status bits (1: line
                          search cap, 4: team barrier timed out, 8: no positive
                          entry in flux/(flux+bkg)*AT(gn), where the reference
                          raises, sgp.py:269-270), trials evaluated
                          from the small-step series, team size T, projection
                          passes over the image, projection-list entries read;
                          may be NULL */
  double* err;         /* [B][MAXIT1] relative error ||x_k - obj|| / ||obj|| of the
                          scaled iterate after the initial projection (k = 0) and after
                          iteration k (errflag, sgp.py:240-257, 394-396); needs in->obj;
                          may be NULL */
  double* x_iter;      /* [B][MAXIT][H][W] the scaled iterate after each iteration,
                          before the revert (save=True writes these, sgp.py:416-422);
                          may be NULL */
} bsgp_outputs;

/* Plan: geometry, FFT sizes, twiddles and the PSF transfer functions for A and
 * AT, built on the device from the host PSF [kh][kw].  storage: BSGP_STORAGE_F64,
 * or BSGP_STORAGE_F32 (iteration vectors kept in float32 in HBM, every sum and
 * scalar in float64; SURVEY config C4).  Synchronous. */
int bsgp_plan_create(int32_t H, int32_t W, const double* psf_host, int32_t kh, int32_t kw,
                     int32_t conv_mode, int32_t storage, int32_t device, bsgp_plan* out);
/* The same; psf_checked != 0 skips the normalisation check because the caller
 * has applied the reference's check (sgp.py:97-102 / 557-562: np.sum in the
 * PSF's OWN dtype) before widening the PSF to float64 -- a float32 PSF whose
 * float32 sum is 1 has a float64 sum off by up to ~1e-7, which the float64
 * check here would refuse.  The Python drop-in always checks first. */
int bsgp_plan_create_checked(int32_t H, int32_t W, const double* psf_host, int32_t kh,
                             int32_t kw, int32_t conv_mode, int32_t storage, int32_t device,
                             int32_t psf_checked, bsgp_plan* out);
int bsgp_plan_destroy(bsgp_plan plan);
/* FFT grid (P x Q) and the per-slot workspace bytes of the plan. */
int bsgp_plan_info(bsgp_plan plan, int32_t* P, int32_t* Q, int64_t* slot_bytes,
                   int32_t* fft_waves);

/* Batched SGP / beta-SGP: B independent images (or (image, beta) candidates),
 * each solved to completion by one persistent workgroup. Asynchronous. */
int bsgp_solve_device(bsgp_plan plan, int32_t B, const bsgp_params* params,
                      const bsgp_inputs* in, const bsgp_outputs* out, void* stream);

/* Measurement: bsgp_solve_device on the one stream `stream` (params->streams is
 * taken as 1) with a HIP event recorded around every kernel launch;
 * kernel_ms[k] and launches[k] (k < 6) receive the summed span and the launch
 * count of kernel class k: 0 setup, 1 k_dir, 2 k_col (A and AT), 3 k_ls, 4 k_bb,
 * 5 k_persist (the persistent solver: every iteration in one launch).
 * Synchronous (waits for the solve). */
int bsgp_solve_profiled(bsgp_plan plan, int32_t B, const bsgp_params* params,
                        const bsgp_inputs* in, const bsgp_outputs* out, void* stream,
                        double* kernel_ms, int64_t* launches);

/* Same with host buffers (copies in, solves, copies out). Synchronous. */
int bsgp_solve_host(bsgp_plan plan, int32_t B, const bsgp_params* params,
                    const bsgp_inputs* in, const bsgp_outputs* out);

/* A (transpose=0) or AT (transpose=1) of the plan on B images. Asynchronous.
 * Replaces the partial(afunction/A/AT, ...) operators of sgp.py:119-120,160-161. */
int bsgp_apply_operator(bsgp_plan plan, int32_t B, int32_t transpose, const double* x,
                        double* out, void* stream);

/* flux_conserve_proj.projectDF(b, c, dia, scaling, ccd_sat_level, lambda_,
 * dlambda_, tol_lam, biter, siter, max_projs) on one vector of length n.
 * x: output [n]; info: output [4] = {final lambda, evaluations, biter, siter}.
 * Asynchronous. */
int bsgp_project_df(int64_t n, double b, const double* c, const double* dia, double scaling,
                    int32_t has_sat, double ccd_sat_level, double lambda0, double dlambda0,
                    double tol_lam, int32_t biter, int32_t siter, int32_t max_projs, double* x,
                    double* info, void* stream);

/* betaDiv(y, x, beta) (sgp.py:441-458) -> out[0]. Asynchronous. */
int bsgp_beta_div(int64_t n, const double* y, const double* x, double beta, double* out,
                  void* stream);
/* betaDivDeriv(y, x, beta) elementwise (sgp.py:462-495) -> out[n]. Asynchronous. */
int bsgp_beta_div_deriv(int64_t n, const double* y, const double* x, double beta, double* out,
                        void* stream);
/* The two elementwise parts of betaDivDerivwrtY (sgp.py:498-499):
 * pow1 = den**(beta-1), w = gn*den**(beta-2). Asynchronous. */
int bsgp_beta_div_grad_parts(int64_t n, const double* den, const double* gn, double beta,
                             double* pow1, double* w, void* stream);

/* ---- data paths either side of the solver ---------- */

/* Overlapping subdivision tiles of an [H][W] field: out[t] = img[y0:y1, x0:x1]
 * for boxes[t] = {x0, y0, x1, y1} (device int32 [n][4], xyxy as
 * restoration/utils.py:332-372 calculate_slice_bboxes returns them), every
 * box exactly th x tw and inside the field.  Replaces create_subdivisions'
 * Cutout2D cutouts (utils.py:375-386).  Asynchronous. */
int bsgp_extract_tiles(const double* img, int32_t H, int32_t W, const int32_t* boxes, int32_t n,
                       int32_t th, int32_t tw, double* out, void* stream);

/* Mean co-add of n th x tw tiles at boxes into an [H][W] mosaic; footprint
 * (may be NULL) = number of tiles covering each pixel; uncovered pixels are 0.
 * Tiles are summed in index order (deterministic).  The same-WCS case of
 * reproject_and_coadd (utils.py:389-395) with combine_function='mean' and no
 * background matching.  n <= 8192.  Asynchronous. */
int bsgp_coadd_tiles(const double* tiles, int32_t n, int32_t th, int32_t tw, const int32_t* boxes,
                     int32_t H, int32_t W, double* mean, double* footprint, void* stream);

/* FITS primary-array samples (big-endian, BITPIX 8/16/32/64/-32/-64) to f64:
 * out[i] = BZERO + BSCALE * sample[i] (FITS standard 4.0 §5.3; IEEE samples
 * exact).  raw: device copy of the data block, 8-byte aligned.  Replaces
 * astropy.io.fits reads of the results/ and psf/ FITS files.  Asynchronous. */
int bsgp_fits_to_f64(const void* raw, int64_t n, int32_t bitpix, double bscale, double bzero,
                     double* out, void* stream);

/* DIAPL PSF model: the values of a psf*.bin.txt coefficient file
 * (psf/psf_calculate.py:10-47 reads them in this order) plus the degrees the
 * reference evaluates with (ldeg = 2, sdeg = 1: psf_calculate.py:24-25). */
typedef struct {
  int32_t hw;            /* stamp half width: stamps are (2hw+1) x (2hw+1)  (value 0) */
  int32_t ngauss;        /* Gaussian components                           (value 3) */
  int32_t ldeg;          /* local polynomial degree of calc_psf_pix (self.ldeg) */
  int32_t sdeg;          /* spatial polynomial degree of init_psf (self.sdeg) */
  double cos, sin;       /* values 5-6 */
  double ax, ay;         /* values 7-8 */
  double sigma_inc;      /* value 9 */
  double x_orig, y_orig; /* values 12-13: origin of the spatial expansion */
  const double* coeffs;  /* host: values 14.. (ngauss*(ldeg+1)(ldeg+2)/2 per spatial term) */
  int32_t ncoef;
} bsgp_psf_model;

/* n PSF stamps [n][2hw+1][2hw+1] (device out).  spatial = 0: the local
 * coefficients are coeffs[0:ncomp] for every stamp (get_psf_mat,
 * psf_calculate.py:89-107; xy may be NULL); spatial = 1: the coefficients at
 * field position xy[2i], xy[2i+1] (device, (x, y)) by the spatial expansion of
 * init_psf (:140-165).  normalize = 1 divides each stamp by its numpy-order sum
 * (normalize_psf_mat, :129-137).  Pixel (r, c) is calc_psf_pix(x = c - hw,
 * y = r - hw) (:98-103).  Asynchronous. */
int bsgp_psf_stamps(const bsgp_psf_model* model, const double* xy, int32_t n, int32_t spatial,
                    int32_t normalize, double* out, void* stream);

/* Per-image PSFs: replace the plan's transfer functions with n pairs built on
 * the device from device PSF stamps [n][kh][kw] (the kh x kw the plan was
 * created with; H x W in circular mode), each checked like sgp.py:97-102.
 * Afterwards bsgp_solve_* and bsgp_apply_operator on this plan need B == n and
 * image i is convolved with PSF i (the spatially varying PSF of each
 * subdivision).  Synchronous. */
int bsgp_plan_set_psfs(bsgp_plan plan, const double* psfs_dev, int32_t n, void* stream);

int bsgp_device_synchronize(void);
const char* bsgp_last_error(void);
int32_t bsgp_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* BSGP_H_ */

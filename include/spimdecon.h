/*
 * spimdecon.h -- C-ABI of libspimdecon.so, the MI355X-native drop-in for the
 * multiview Richardson-Lucy deconvolution + DoG bead-detection hot path of
 * PreibischLab/SPIM_Registration.
 *
 * Reference interfaces replaced (paths under /root/reference/src/main/java/):
 *   - spim/process/cuda/CUDAFourierConvolution.java:4-10      (FourierConvolutionCUDALib, JNA)
 *   - spim/process/cuda/CUDAStandardFunctions.java:15-23      (device query, JNA)
 *   - spim/process/cuda/CUDASeparableConvolution.java:13-21   (SeparableConvolutionCUDALib, JNA)
 *   - spim/process/fusion/deconvolution/MVDeconvolution.java:73-444 (RL loop; new session API)
 *   - spim/process/fusion/deconvolution/MVDeconFFT.java:162-303     (kernel preparation)
 *   - spim/process/interestpointdetection/ProcessDOG.java:40-178    (DoG pass)
 *
 * Conventions
 *   - Plain C types only; every pointer is caller-owned and only read/written
 *     during the call.  Volumes are x-fastest float32 (ImgLib2 ArrayImg order).
 *   - JNA type mapping: Java boolean -> int32_t, Java long -> int64_t,
 *     float[]/int[] -> pointers (JNA copies arrays in and back out).
 *   - Status codes: 0 = OK, negative = error; the message of the last error of
 *     the calling thread is returned by spimdecon_last_error().
 *   - No CPU fallback: a negative/invalid device id or a missing GPU is an
 *     error (status SPIMDECON_ERR_DEVICE), never a silent CPU path.
 */
#ifndef SPIMDECON_H
#define SPIMDECON_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPIMDECON_OK               0
#define SPIMDECON_ERR_ARG         -1
#define SPIMDECON_ERR_DEVICE      -2
#define SPIMDECON_ERR_HIP         -3
#define SPIMDECON_ERR_FFT         -4
#define SPIMDECON_ERR_COMM        -5
#define SPIMDECON_ERR_STATE       -6
#define SPIMDECON_ERR_OOM         -7
#define SPIMDECON_ERR_IO          -8   /* file cannot be opened (Java: IOException) */

/* last error message of the calling thread ("" if none) */
const char* spimdecon_last_error(void);
/* library version string, e.g. "spimdecon 0.1.0 gfx950 rocfft 1.0.36" */
const char* spimdecon_version(void);

/* ======================================================================
 * 1. Legacy FourierConvolutionCUDALib ABI
 *    spim/process/cuda/CUDAFourierConvolution.java:9-10; called from
 *    spim/process/fusion/deconvolution/MVDeconFFTThreads.java:65-68,88-91.
 * ====================================================================== */

/* In-place circular 3D convolution of one block with a kernel whose centre
 * kernelDim/2 is moved to the origin (the block already carries the K-1 halo).
 * imDim / kernelDim are REVERSED: {nz, ny, nx} (MVDeconFFTThreads.java:136-144).
 * Thread-safe: one Java thread per device calls this concurrently
 * (MVDeconFFT.java:424-446); per-device plan and stream caches.
 * Java declares `void`; the int status is ignored by such a binding. */
int convolution3DfftCUDAInPlace(float* im, const int* imDim,
                                const float* kernel, const int* kernelDim,
                                int devCUDA);

/* Out-of-place variant (declared at CUDAFourierConvolution.java:9, never
 * called by the reference).  Returns a buffer owned by the library that must
 * be released with spimdecon_free(); NULL on error. */
float* convolution3DfftCUDA(const float* im, const int* imDim,
                            const float* kernel, const int* kernelDim,
                            int devCUDA);
void spimdecon_free(void* p);

/* ======================================================================
 * 2. Device query ABI -- spim/process/cuda/CUDAStandardFunctions.java:15-23,
 *    consumer spim/process/cuda/CUDATools.java:35-192.
 * ====================================================================== */
int     getNumDevicesCUDA(void);                       /* -1 = driver error, 0 = none */
void    getNameDeviceCUDA(int devCUDA, char* name);    /* name: >= 256 bytes */
int64_t getMemDeviceCUDA(int devCUDA);
int64_t getFreeMemDeviceCUDA(int devCUDA);
/* gfx950 is reported as "compute capability" 9.5 (major 9, minor 5) */
int     getCUDAcomputeCapabilityMajorVersion(int devCUDA);
int     getCUDAcomputeCapabilityMinorVersion(int devCUDA);

/* ======================================================================
 * 3. SeparableConvolutionCUDALib ABI -- spim/process/cuda/CUDASeparableConvolution.java:13-17;
 *    caller spim/process/cuda/CUDASeparableConvolutionFunctions.java:176-196.
 *    In-place separable convolution of a w*h*d x-fastest image with centred
 *    kernels of length N (7/15/31/63/127).  Dims NOT reversed.
 *    outofbounds: 0 = zero, 1 = value (outofboundsvalue), 2 = extend border
 *    pixel; 3 = mirror-single (extension used by this library's DoG pass).
 *    Returns 1 (Java true) on success, 0 on failure.
 * ====================================================================== */
int32_t convolve_7  (float* image, const float* kernelX, const float* kernelY, const float* kernelZ,
                     int imageW, int imageH, int imageD, int32_t convolveX, int32_t convolveY,
                     int32_t convolveZ, int outofbounds, float outofboundsvalue, int devCUDA);
int32_t convolve_15 (float* image, const float* kernelX, const float* kernelY, const float* kernelZ,
                     int imageW, int imageH, int imageD, int32_t convolveX, int32_t convolveY,
                     int32_t convolveZ, int outofbounds, float outofboundsvalue, int devCUDA);
int32_t convolve_31 (float* image, const float* kernelX, const float* kernelY, const float* kernelZ,
                     int imageW, int imageH, int imageD, int32_t convolveX, int32_t convolveY,
                     int32_t convolveZ, int outofbounds, float outofboundsvalue, int devCUDA);
int32_t convolve_63 (float* image, const float* kernelX, const float* kernelY, const float* kernelZ,
                     int imageW, int imageH, int imageD, int32_t convolveX, int32_t convolveY,
                     int32_t convolveZ, int outofbounds, float outofboundsvalue, int devCUDA);
int32_t convolve_127(float* image, const float* kernelX, const float* kernelY, const float* kernelZ,
                     int imageW, int imageH, int imageD, int32_t convolveX, int32_t convolveY,
                     int32_t convolveZ, int outofbounds, float outofboundsvalue, int devCUDA);

/* CPU variant declared by the same interface (CUDASeparableConvolution.java:21) and
 * never called by the reference.  There is no CPU path here: returns
 * SPIMDECON_ERR_DEVICE and leaves the image unchanged (a `void` JNA binding ignores
 * the status; spimdecon_last_error() holds the message). */
int     convolutionCPU(float* image, const float* kernelX, const float* kernelY, const float* kernelZ,
                       int kernelRX, int kernelRY, int kernelRZ, int imageW, int imageH, int imageD,
                       int outofbounds, float outofboundsvalue);

/* ======================================================================
 * 4. Kernel preparation -- spim/process/fusion/deconvolution/MVDeconFFT.java:162-303
 *    (MVDeconInput.init order, AdjustInput.normImg quirk with ij_threads).
 * ====================================================================== */
#define MVD_PSF_OPTIMIZATION_II     0   /* MVDeconFFT.PSFTYPE ordinals, MVDeconFFT.java:28 */
#define MVD_PSF_OPTIMIZATION_I      1
#define MVD_PSF_EFFICIENT_BAYESIAN  2
#define MVD_PSF_INDEPENDENT         3

/* kdims: 3*nviews ints, per view {kx, ky, kz} (odd).  k1_out[v] receives the
 * normalised kernel1, k2_out[v] kernel2 (both kx*ky*kz floats).  Runs on GPU
 * devCUDA. */
int mvd_prepare_kernels(int nviews, const float* const* k1_in, const int* kdims,
                        int psftype, int ij_threads,
                        float* const* k1_out, float* const* k2_out, int devCUDA);

/* out[i] = MVDeconvolution.computeNextValue(last[i], integral[i], weight[i])
 * (MVDeconvolution.java:671-703; lambda > 0: the Tikhonov branch :681-690) for
 * n voxels, DEVICE pointers on the current device -- the exact per-voxel rule the
 * session's update step applies, exposed so callers and tests can check it bit for
 * bit against the reference rule.  Synchronous. */
int spimdecon_next_value(const float* last, const float* integral, const float* weight, int64_t n,
                         double lambda, float* out);

/* ======================================================================
 * 5. GPU-resident RL session (replaces MVDeconvolution.runIteration's
 *    per-view convolve1 -> quotient -> convolve2 -> update loop,
 *    MVDeconvolution.java:333-444, and the init/mask of :95-187).
 * ====================================================================== */
typedef struct mvd_session mvd_session;

typedef struct mvd_params {
    int64_t dims[3];        /* {nx, ny, nz} of THIS rank's z-range of psi          */
    int64_t nz_global;      /* global nz (== dims[2] for a single rank)            */
    int64_t z_offset;       /* first global z plane owned by this rank             */
    int     device;         /* HIP device id (>= 0)                                */
    int     local_slabs;    /* z-slabs held by this process (>= 1); >1 = virtual shards */
    int     nranks;         /* processes in the RCCL communicator (1: none unless comm_id) */
    int     rank;
    const char* comm_id;    /* 128-byte RCCL unique id (required when nranks > 1;
                               with nranks == 1 a non-NULL id still makes a one-rank
                               communicator: collectives and watchdog through RCCL) */
    int     storage_fp16;   /* 1: img/weights stored as fp16 (config-5 mode)       */
    int     fft_pad_policy; /* padded FFT length per axis (>= n + K - 1):            *
                             * 0 = auto (two-factor fast-path length when within    *
                             *     25% of the smallest 2,3,5,7-smooth length),      *
                             * 1 = fast-path table only, 2 = smallest smooth length */
    int     halo[3];        /* max kernel half size {cx,cy,cz}; 0 = derive from views */
    int     ij_threads;     /* pinned reference thread count for the normImg quirk  */
    int     fft_backend;    /* 0 = fused spectral engine (default), 1 = rocFFT       */
    int     slab_axis;      /* axis the volume is split along (local slabs, devices,  *
                             * ranks): 0 = z (default), 1 = y, -1 = the longer of y  *
                             * and z when the volume is split (one rank; else z).    *
                             * With y, dims is this rank's                           *
                             * y-range of every z plane and nz_global / z_offset     *
                             * give the global ny / first y row; the session keeps   *
                             * its slabs in (x, z, y) order internally (one row      *
                             * transposition at upload / download)                   */
    int     reserved[6];
} mvd_params;

/* fills *p with defaults (local_slabs=1, nranks=1, ij_threads=8, ...) */
void mvd_params_default(mvd_params* p);

/* 128-byte RCCL unique id for rank 0 to broadcast (torch.distributed / MPI) */
int mvd_comm_unique_id(char* out128);

/* global [z0, z1) of part `idx` of `nparts` over nz planes (balanced split) */
int mvd_slab_range(int64_t nz, int nparts, int idx, int64_t* z0, int64_t* z1);

/* The halo transfers of one slab (nz interior planes, Mz padded planes, cz halo planes,
 * plane_elems floats per padded plane), as float offsets into its spectrum buffer:
 * out5 = {send_lo, recv_lo, send_hi, recv_hi, count}.  To / from the lower neighbour:
 * send [0, cz), receive into [Mz - cz, Mz); to / from the upper one: send [nz - cz, nz),
 * receive into [nz, nz + cz).  The one helper behind the local slab copies, the device-
 * group peer pulls and the RCCL send / recv (MVDeconFFT.java:424-446 runs the blocks of
 * one volume on several devices; here neighbouring slabs trade halo planes). */
int mvd_halo_plan(int64_t nz, int64_t Mz, int cz, int64_t plane_elems, int64_t* out5);

int  mvd_create(const mvd_params* params, mvd_session** out);
/* One session over several GPUs of this process -- the reference's
 * MVDeconFFT(img, weight, kernel, factory, int[] deviceList, ...) driven from one
 * JVM (MVDeconFFT.java:58-64,91-100,424-446).  params.dims is the whole
 * (this rank's) volume; it is split into ndev * params.local_slabs z-slabs, slabs
 * [i*local_slabs, (i+1)*local_slabs) on devs[i] (params.device is ignored).  One
 * mvd_run drives all devices (one host thread each); halo planes move between
 * neighbouring devices as peer copies over xGMI.  Device ids may repeat (several
 * groups on one GPU: the same code path, e.g. for testing).  Needs the engine
 * backend and nranks == 1. */
int  mvd_create_devices(const int* devs, int ndev, const mvd_params* params, mvd_session** out);
void mvd_destroy(mvd_session* h);
/* devices of the session and the device holding slab s (slabs: ndev * local_slabs) */
int  mvd_num_devices(mvd_session* h, int* ndev);
int  mvd_slab_device(mvd_session* h, int slab, int* dev);
/* slabs of the session: ndev * local_slabs, where local_slabs may exceed
 * params.local_slabs -- the engine splits a device's share further until every
 * slab buffer (psi, views, spectra) stays below 4 GiB, the range of its 32-bit
 * buffer offsets (env SPIMDECON_AUTO_SLABS=0 disables; the slabs are exact, like
 * the reference's precise blocks, BlockGeneratorFixedSizePrecise.java:25-101) */
int  mvd_num_slabs(mvd_session* h, int* nslabs);
/* voxels {nx, ny, nz} of slab s in the session's internal order (a y-split session
 * keeps (x, z, y-slab) rows: nz is then the slab's y extent) */
int  mvd_slab_extent(mvd_session* h, int slab, int64_t* out3);
/* halo exchange counters since mvd_create: bytes and copies moved between slabs
 * (local copies, peer pulls between device groups, RCCL sends); either may be NULL */
int  mvd_exchange_stats(mvd_session* h, int64_t* bytes, int64_t* copies);

/* Adds one view (MVDeconInput.add order).  img/weight: this rank's z-range,
 * dims = params.dims; kernel1: raw (un-normalised) PSF of kdims {kx,ky,kz}.
 * Views are only staged here; mvd_init() builds kernels and uploads. */
int mvd_add_view(mvd_session* h, const float* img, const float* weight,
                 const float* kernel1, const int* kdims);
/* Same, but img/weight are device pointers on params.device (copied). */
int mvd_add_view_device(mvd_session* h, const float* d_img, const float* d_weight,
                        const float* kernel1, const int* kdims);

/* MVDeconInput.init(type): normalises kernel1 and builds kernel2 for all
 * views (MVDeconFFT.java:162-303) then computes the kernel spectra. */
int mvd_init(mvd_session* h, int psftype);
/* Alternative to mvd_init: kernels already prepared by the caller
 * (MVDeconFFT.getKernel1/2, MVDeconFFT.java:352-353). */
int mvd_set_kernels(mvd_session* h, int view, const float* k1, const float* k2);
/* read back prepared kernels (kx*ky*kz floats each) */
int mvd_get_kernels(mvd_session* h, int view, float* k1, float* k2);

/* psi initialisation (MVDeconvolution.java:95-127).  psi == NULL: first-iteration
 * average fusion (FirstIteration.java, NaN -> 0.5); else the given image with
 * the checkNumbers clamp (<= 0 -> minValue). *avg_out may be NULL. */
int mvd_init_psi(mvd_session* h, const float* psi_or_null, double* avg_out);

/* runs `iters` RL iterations (sequential per-view updates).  lambda > 0:
 * Tikhonov.  stats (may be NULL): iters*nviews*2 doubles {sumChange, maxChange}
 * reduced over all slabs and ranks. */
int mvd_run(mvd_session* h, int iters, double lambda, double* stats);

/* final mask: psi = 0 where no view has data (MVDeconvolution.java:180-187) */
int mvd_apply_mask(mvd_session* h);

/* copy this rank's psi to out (dims of params); out may be a host or a device
 * pointer (unified addressing: a device-resident result skips the host) */
int mvd_get_psi(mvd_session* h, float* out);
/* device pointer of local slab s's psi (valid until mvd_destroy); x-fastest
 * [z][y][x] of the slab, or [y][z][x] when the session splits along y */
float* mvd_psi_device(mvd_session* h, int slab);

/* padded FFT dims {Mx, My, Mz} of local slab s (info/bench) */
int mvd_fft_dims(mvd_session* h, int slab, int64_t* out3);
/* z-planes of each stored kernel spectrum (info/bench): 2*cz+1 when the engine
 * keeps compact kernels (the z pass builds their z transform), else Mz */
int mvd_kernel_planes(mvd_session* h, int slab, int* planes);
/* z pass of the engine (info/bench): 0 = fused FFT z pass with full kernel
 * spectra, 1 = fused FFT z pass with compact kernels, 3 = direct circular
 * convolution with the compact kernel over z chunks carried inside a block (only
 * the nz interior planes written; 2 and 4 named passes removed in round 5);
 * -1 for the rocFFT backend */
int mvd_zpass_mode(mvd_session* h, int slab, int* mode);
/* x pass of the last update launch of slab s (info/tests): 2 = two-factor row-pair
 * tiles, 1 = per-wave rows, 0 = Stockham rows, -1 = no run yet, -2 = rocFFT backend */
int mvd_xpass_mode(mvd_session* h, int slab, int* mode);
/* HIP stream the session launches on (hipStream_t as void*) */
void* mvd_stream(mvd_session* h);
/* per-kernel timing: when enabled, mvd_run records HIP events around every
 * kernel class; mvd_timing fills out16[0..7] with the accumulated ms and
 * out16[8..15] with the launch count of each class:
 *   engine backend: [0] x update pass, [1] x quotient pass, [2] y passes,
 *                   [3] z convolve passes, [4] psi forward x pass,
 *                   [5] halo exchange, [6] stats reduce
 *   rocFFT backend: [0] update + pad, [1] quotient + pad, [2] R2C,
 *                   [3] spectral multiply, [4] C2R, [5] halo exchange,
 *                   [6] stats reduce */
int mvd_enable_timing(mvd_session* h, int on);
int mvd_timing(mvd_session* h, double* out16);

/* ======================================================================
 * 6. DoG bead detection -- spim/process/interestpointdetection/ProcessDOG.java:40-178
 * ====================================================================== */
typedef struct spim_dog_params {
    float   sigma;           /* default 1.8 (DifferenceOfGaussian.java:36)          */
    float   threshold;       /* default 0.008 (DifferenceOfGaussian.java:37)        */
    int     localization;    /* 0 = none (threshold), 1 = quadratic (threshold/10)  */
    double  image_sigma[3];  /* default 0.5 each; min(imageSigma, sigma) applied    */
    int32_t find_min;
    int32_t find_max;
    double  min_intensity;   /* NaN -> image min/max                                */
    double  max_intensity;
    int     ij_threads;      /* peak ordering: lists by x % T (InteractiveIntegral.java:394) */
    int     device;
} spim_dog_params;

typedef struct spim_peak {
    int32_t x, y, z;
    float   intensity;       /* |dog| */
    int32_t is_min, is_max;
} spim_peak;

/* InterestPoint(Value) of spim.fiji.spimdata.interestpoints (id = index) */
typedef struct spim_interest_point {
    double  pos[3];          /* x, y, z (sub-pixel with localization 1)             */
    float   intensity;       /* |dog| (localization 0) or the fitted value (1)       */
    int32_t is_max;
} spim_interest_point;

void spim_dog_params_default(spim_dog_params* p);

/* img: dims {nx, ny, nz} x-fastest (not modified).  dog_out (optional, may be
 * NULL) receives the DoG image.  img and dog_out may be host or device (HIP)
 * pointers: a view already resident in HBM is not staged through the host.  peaks: capacity max_peaks, *npeaks = total
 * found (may exceed max_peaks: then only max_peaks were written).  These are
 * the DoG extrema with |v| >= threshold (localization 0) or threshold / 10
 * (localization 1), i.e. DifferenceOfGaussianNewPeakFinder.getSimplePeaks. */
int spim_dog_compute(const float* img, const int64_t* dims, const spim_dog_params* p,
                     float* dog_out, spim_peak* peaks, int64_t max_peaks, int64_t* npeaks);

/* ProcessDOG.compute's result (ProcessDOG.java:150-168): the peaks above
 * after Localization -- localization 0: Localization.noLocalization
 * (Localization.java:19-45); 1: quadratic sub-pixel fit, kept when
 * |fitted value| > threshold (Localization.java:47-88).  Same capacity rule
 * as spim_dog_compute. */
int spim_dog_interest_points(const float* img, const int64_t* dims, const spim_dog_params* p,
                             float* dog_out, spim_interest_point* out, int64_t max_out,
                             int64_t* nout);

/* The two DoG calls above keep a per-device workspace between calls (the
 * intermediate Gaussians, candidate lists; ~12 B per voxel of the largest view seen)
 * instead of allocating per call; this frees it.  No reference counterpart (the
 * reference's CUDA library allocates per call, CUDASeparableConvolution.java:13-21). */
int spim_dog_release_workspace(int device);

/* Interest-point list files (InterestPointList.java:66-100 save, :178-220 load):
 * <base_dir>/<file>.ip.txt (base_dir may be NULL or ""; missing parent directories
 * are created), header "id\tx\ty\tz", one line per point with the doubles printed
 * as Java's Double.toString.  ids (may be NULL: id = index, as ProcessDOG assigns
 * them) are written / read beside pos.  Load: *nout = points in the file; at most
 * max_out are stored (intensity / is_max are 0: the file holds positions only). */
int spim_save_interest_points(const char* base_dir, const char* file, const spim_interest_point* pts,
                              const int32_t* ids, int64_t n);
int spim_load_interest_points(const char* base_dir, const char* file, spim_interest_point* out,
                              int32_t* ids, int64_t max_out, int64_t* nout);
/* Java Double.toString of d into out (cap bytes incl. the terminator), in the form of
 * the selected Java version (also used by spim_save_interest_points): 8 (default; Fiji
 * runs Java 8: sun.misc.FloatingDecimal, e.g. 2.0E23 -> "1.9999999999999998E23") or 19
 * (JDK 19+: the shortest decimal that round-trips, "2.0E23").  Process-wide. */
int spim_set_java_version(int jdk);
int spim_java_double_to_string(double d, char* out, int cap);

/* ======================================================================
 * 7. Deconvolution input preparation --
 *    spim/process/fusion/deconvolution/ProcessForDeconvolution.java:159-384:
 *    each view resampled into the fused bounding box through the inverse of
 *    its affine model (TransformInput(AndWeights)), cosine blending weights,
 *    WeightNormalizer, OSEM adjustment.
 * ====================================================================== */
#define SPIM_WEIGHTS_NONE         0   /* WeightType.NO_WEIGHTS                          */
#define SPIM_WEIGHTS_PRECOMPUTED  1   /* WeightType.PRECOMPUTED_WEIGHTS                 */
#define SPIM_WEIGHTS_VIRTUAL      2   /* WeightType.VIRTUAL_WEIGHTS (the default)       */

typedef struct spim_view_source {
    const float* img;        /* source stack, x-fastest {nx, ny, nz}                     */
    int64_t      dims[3];
    double       model[12];  /* row-major 3x4 affine, source -> world (ViewRegistration)  */
} spim_view_source;

typedef struct spim_input_params {
    int64_t bb_min[3];           /* bounding box of the fused volume (world voxels)       */
    int64_t bb_dims[3];
    float   blending_border[3];  /* default -8 (EfficientBayesianBased.java:76)          */
    float   blending_range[3];   /* default 12 (EfficientBayesianBased.java:75)           */
    int     weight_type;         /* SPIM_WEIGHTS_*                                         */
    int     osem_index;          /* 0: osem_speedup, 1: min, 2: average overlapping views  */
    double  osem_speedup;
    int     ij_threads;          /* portions of the overlap statistics (2T)               */
    int     device;
    int     src_on_device;       /* 1: views[].img are device pointers                    */
    int     out_on_device;       /* 1: img_out / weight_out are device pointers           */
    int     reserved[8];
} spim_input_params;

void spim_input_params_default(spim_input_params* p);

/* img_out[v], weight_out[v]: bb_dims voxels each (x-fastest).  osem_used,
 * min_overlap, avg_overlap (may be NULL) report the OSEM factor applied and
 * WeightNormalizer's overlap statistics (-1 / NaN for SPIM_WEIGHTS_NONE). */
int spim_prepare_inputs(int nviews, const spim_view_source* views, const spim_input_params* p,
                        float* const* img_out, float* const* weight_out, double* osem_used,
                        int* min_overlap, double* avg_overlap);

/* ======================================================================
 * 8. Weighted-average fusion --
 *    spim/process/fusion/weightedavg/ProcessParalellPortion(Weight).java:
 *    per fused voxel the (blending-weighted) mean of the views covering it.
 * ====================================================================== */
typedef struct spim_fusion_params {
    int64_t bb_min[3];      /* bounding box (world voxels)                               */
    int64_t bb_dims[3];     /* fused image dims (after downsampling)                    */
    float   downsampling;   /* 1 = none; s = position * downsampling + bb_min            */
    int     interpolation;  /* 0 nearest neighbour, 1 n-linear (Fusion.defaultInterpolation) */
    int     use_blending;   /* Fusion.defaultUseBlending (content-based not supported)  */
    int     device;
    int     src_on_device;
    int     out_on_device;
    int     reserved[8];
} spim_fusion_params;

void spim_fusion_params_default(spim_fusion_params* p);

/* blending_borders / blending_ranges: 3 floats per view (may be NULL without
 * blending); out: bb_dims voxels, x-fastest float32. */
int spim_fuse_weighted_average(int nviews, const spim_view_source* views, const spim_fusion_params* p,
                               const float* blending_borders, const float* blending_ranges, float* out);

/* ======================================================================
 * 9. PSF extraction / transformation --
 *    spim/process/fusion/deconvolution/ExtractPSF.java.  All buffers are
 *    x-fastest float32 in host memory unless stated; dims are (x, y, z).
 * ====================================================================== */

/* transformPSF (:309-346): odd size of the transformed PSF and the offset that
 * keeps model(dim / 2) at its centre voxel (offset may be NULL). */
int spim_psf_transformed_size(const int64_t psf_size[3], const double model[12], int64_t out_size[3],
                              double offset[3]);

/* transformPSF + transform (:309-346, :424-460): n-linear over a zero-extended
 * PSF at inverse(model)(i + offset); out holds spim_psf_transformed_size voxels.
 * Also the path of loadAndTransformPSFs (:520-575) for PSFs read from files. */
int spim_transform_psf(const float* psf, const int64_t psf_size[3], const double model[12], float* out,
                       int device);

/* extractNextImg (:260-279): extractPSFLocal (:383-422; the sum over beads of
 * the n-linear samples of the periodic-extended view at i - size/2 + bead,
 * locations = nlocations x (x, y, z) local pixel coordinates), normalize
 * (:281-299) into psf_original (psf_size voxels), then -- when psf_transformed
 * is not NULL -- transformPSF with the view model.  img may be a device
 * pointer (img_on_device = 1), e.g. the source stack of spim_prepare_inputs. */
int spim_extract_psf(const float* img, const int64_t dims[3], int img_on_device, const double* locations,
                     int64_t nlocations, const int64_t psf_size[3], const double model[12], float* psf_original,
                     float* psf_transformed, int device);

/* spim_extract_psf for nviews views at once (ExtractPSF.extract over the views of a
 * timepoint): dims, models are nviews x 3 / x 12 (models may be NULL when
 * psf_transformed is NULL; entries of psf_transformed may be NULL); psf_original
 * and psf_transformed entries may be host or device pointers.  The views run
 * concurrently on their own streams: one view's bead sum is psf_size serial float
 * chains (bead order, as the reference), too few to fill the GPU alone.  Results are
 * identical to nviews spim_extract_psf calls. */
int spim_extract_psfs(int nviews, const float* const* imgs, const int64_t* dims, int img_on_device,
                      const double* const* locations, const int64_t* nlocations, const int64_t psf_size[3],
                      const double* models, float* const* psf_original, float* const* psf_transformed,
                      int device);

/* spim_extract_psf(s) keep one view's device buffers and stream per view between
 * calls (a whole view when img is a host pointer, the bead samples, the PSFs); this
 * frees them on `device` (-1: every device), e.g. before an RL session is created on
 * the same GPU.  No reference counterpart (ExtractPSF allocates per call). */
int spim_psf_release_workspace(int device);

/* computeAverageTransformedPSF (:164-208): the PSFs (psf_dims = npsfs x 3)
 * point-mirrored about their centres and summed into the max size, written
 * to avg_dims.  avg == NULL: only the dims are returned. */
int spim_average_transformed_psf(int npsfs, const float* const* psfs, const int64_t* psf_dims, float* avg,
                                 int64_t avg_dims[3], int device);

/* computeMaxProjection (:110-162): max along min_dim (0 x, 1 y, 2 z; < 0 = the
 * first smallest dimension, returned in used_dim).  out == NULL: dims only. */
int spim_max_projection(const float* img, const int64_t dims[3], int min_dim, float* out, int64_t out_dims[2],
                        int* used_dim, int device);

/* ======================================================================
 * 10. Legacy simultaneous-update multiview RL (opt-in) --
 *     mpicbg/spim/postprocessing/deconvolution/LucyRichardsonMultiViewDeconvolution.java
 *     :24-358 (lucyRichardsonMultiView; LucyRichardsonFFT.java:7-38 holds one view).
 *     Every view's correction is computed from the same psi (not MVDeconvolution's
 *     sequential rule, section 5), so the views shard over ranks -- view v on rank
 *     v % nranks, as the reference hands view v to thread v % numThreads (:127-128) --
 *     and the per-voxel merge of the corrections is one RCCL all-reduce of a double
 *     per voxel each iteration (a product when multiplicative, else a sum).  Every
 *     rank holds the whole psi; all ranks return the same psi and statistics.
 *     The convolutions extend their input by mirroring (extendMirrorSingle): the
 *     reference's imglib1 FourierConvolution is absent and its extension not restated.
 * ====================================================================== */
typedef struct lrsim_session lrsim_session;

/* dims {nx, ny, nz} of the whole volume; nranks > 1 needs the 128-byte comm_id of
 * mvd_comm_unique_id (a non-NULL id with nranks == 1 makes a one-rank communicator) */
int  lrsim_create(const int64_t* dims, int device, int nranks, int rank, const char* comm_id,
                  lrsim_session** out);
/* One process, several GPUs (the reference's threads, LRMV:118-178): view v goes to
 * devs[v % ndev] (ids may repeat); each device holds a psi replica and its views' partial,
 * merged on devs[0] over xGMI each iteration (a sum or a product, in device order), and
 * the new psi copied back.  No RCCL. */
int  lrsim_create_devices(const int64_t* dims, const int* devs, int ndev, lrsim_session** out);
void lrsim_destroy(lrsim_session* h);
/* Adds view number <views so far> (the data list order of the reference).  Every rank
 * adds every view; kdims (odd {kx, ky, kz}) is always required, img / weight / kernel
 * (raw PSF; normImage'd at init) only for the views this rank owns -- NULL otherwise.
 * img / weight: dims voxels, host or device pointers.  Weights are required: the
 * reference's normAllImages reads one per view (:401). */
int  lrsim_add_view(lrsim_session* h, const float* img, const float* weight, const float* kernel,
                    const int* kdims);
int  lrsim_owns_view(lrsim_session* h, int view, int* owned);
/* device holding view `view` on this rank (-1: another rank's view) */
int  lrsim_view_device(lrsim_session* h, int view, int* device);
/* normImage of every kernel (:45-58, exact sum as BigDecimal), psi = (float) the
 * average intensity where two or more views overlap (normAllImages :360-457) */
int  lrsim_init(lrsim_session* h, double* avg_out);
/* iters iterations (the reference's do-while runs max(1, maxIterations)); stats (may be
 * NULL): iters x {sumChange, maxChange} (:309-330).  lambda > 0: Tikhonov (:290-301). */
int  lrsim_run(lrsim_session* h, int iters, int multiplicative, double lambda, double* stats);
/* psi (dims voxels) into a host or device buffer */
int  lrsim_get_psi(lrsim_session* h, float* out);
/* padded FFT lengths {Mx, My, Mz} (info) */
int  lrsim_fft_dims(lrsim_session* h, int64_t* out3);

#ifdef __cplusplus
}
#endif
#endif /* SPIMDECON_H */

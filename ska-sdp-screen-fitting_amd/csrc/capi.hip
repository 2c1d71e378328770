// capi.hip -- the extern "C" boundary of libscreenfit (include/screenfit.h).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "sf_internal.h"

namespace sf {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace sf

using sf::set_error;

namespace {

int check_device(int device) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n == 0) {
    set_error("no HIP device available");
    return SF_ENODEV;
  }
  if (device < 0 || device >= n) {
    set_error("device index out of range");
    return SF_EINVAL;
  }
  hipDeviceProp_t prop;
  SF_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_error(std::string("libscreenfit is built for gfx950, found ") +
              prop.gcnArchName);
    return SF_ENODEV;
  }
  return SF_OK;
}

template <typename T>
int dev_alloc(T** p, size_t count) {
  if (*p) {
    hipFree(*p);
    *p = nullptr;
  }
  if (count == 0) return SF_OK;
  if (hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T)) != hipSuccess) {
    *p = nullptr;
    set_error("hipMalloc failed");
    return SF_ENOMEM;
  }
  return SF_OK;
}

#define SF_TRY(x)              \
  do {                         \
    int rc_ = (x);             \
    if (rc_ != SF_OK) return rc_; \
  } while (0)

}  // namespace

extern "C" {

const char* sf_version(void) { return "screenfit 0.1.0 (gfx950)"; }

const char* sf_last_error(void) { return sf::g_last_error.c_str(); }

int sf_create(int device, sf_ctx** out) {
  SF_REQUIRE(out != nullptr, SF_EINVAL, "sf_create: out is NULL");
  SF_TRY(check_device(device));
  SF_HIP(hipSetDevice(device));
  sf_ctx* ctx = new sf_ctx();
  ctx->device = device;
  if (hipMalloc(reinterpret_cast<void**>(&ctx->d_trash), 1024) != hipSuccess) {
    delete ctx;
    set_error("sf_create: hipMalloc failed");
    return SF_ENOMEM;
  }
  *out = ctx;
  return SF_OK;
}

int sf_destroy(sf_ctx* ctx) {
  if (!ctx) return SF_OK;
  hipSetDevice(ctx->device);
  hipFree(ctx->d_pp);
  hipFree(ctx->d_c);
  hipFree(ctx->d_pinv);
  hipFree(ctx->d_u);
  hipFree(ctx->d_eig);
  hipFree(ctx->d_cfrag);
  hipFree(ctx->d_cdig);
  hipFree(ctx->d_kdig);
  hipFree(ctx->d_kflag);
  if (ctx->kdig_read) (void)hipEventDestroy(ctx->kdig_read);
  hipFree(ctx->d_skip);
  hipFree(ctx->d_st_order);
  hipFree(ctx->d_keys);
  hipFree(ctx->d_ids);
  hipFree(ctx->d_pool_mask);
  hipFree(ctx->d_pool);
  hipFree(ctx->d_pool_status);
  hipFree(ctx->d_pos);
  hipFree(ctx->d_sigma);
  hipFree(ctx->d_class);
  hipFree(ctx->d_counters);
  hipFree(ctx->d_scratch);
  hipFree(ctx->d_wscratch);
  hipFree(ctx->d_oscratch);
  hipFree(ctx->d_gw);
  hipFree(ctx->d_smooth);
  hipFree(ctx->d_tess_tab);
  hipFree(ctx->d_trash);
  delete ctx;
  return SF_OK;
}

int sf_set_stream(sf_ctx* ctx, void* stream) {
  SF_REQUIRE(ctx, SF_EINVAL, "sf_set_stream: NULL context");
  ctx->stream = reinterpret_cast<hipStream_t>(stream);
  return SF_OK;
}

int sf_device_cus(sf_ctx* ctx, int* n_cu) {
  SF_REQUIRE(ctx && n_cu, SF_EINVAL, "sf_device_cus: NULL argument");
  SF_HIP(hipDeviceGetAttribute(n_cu, hipDeviceAttributeMultiprocessorCount,
                               ctx->device));
  return SF_OK;
}

int sf_stream_create(sf_ctx* ctx, const int* reserve_cus, int n_reserve,
                     void** stream) {
  SF_REQUIRE(ctx && stream && n_reserve >= 0 && (n_reserve == 0 || reserve_cus),
             SF_EINVAL, "sf_stream_create: bad argument");
  SF_HIP(hipSetDevice(ctx->device));
  int n_cu = 0;
  SF_TRY(sf_device_cus(ctx, &n_cu));
  hipStream_t s = nullptr;
  if (n_reserve == 0) {
    SF_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  } else {
    std::vector<uint32_t> mask((n_cu + 31) / 32, 0u);
    for (int c = 0; c < n_cu; ++c) mask[c >> 5] |= 1u << (c & 31);
    for (int k = 0; k < n_reserve; ++k) {
      const int c = reserve_cus[k];
      SF_REQUIRE(c >= 0 && c < n_cu, SF_EINVAL, "sf_stream_create: CU index out of range");
      mask[c >> 5] &= ~(1u << (c & 31));
    }
    SF_REQUIRE(n_reserve < n_cu, SF_EINVAL, "sf_stream_create: no CU left");
    SF_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  }
  *stream = s;
  return SF_OK;
}

int sf_stream_destroy(sf_ctx* ctx, void* stream) {
  SF_REQUIRE(ctx && stream, SF_EINVAL, "sf_stream_destroy: bad argument");
  SF_HIP(hipSetDevice(ctx->device));
  SF_HIP(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)));
  return SF_OK;
}

int sf_set_option(sf_ctx* ctx, int option, int value) {
  SF_REQUIRE(ctx, SF_EINVAL, "sf_set_option: NULL context");
  switch (option) {
    case SF_OPT_FIT_GENERAL:
      ctx->force_general = value != 0;
      return SF_OK;
    case SF_OPT_EVAL_KERNEL:
      SF_REQUIRE(value >= SF_EVAL_KERNEL_AUTO && value <= SF_EVAL_KERNEL_SHB,
                 SF_EINVAL, "sf_set_option: unknown evaluation kernel");
      ctx->eval_kernel = value;
      return SF_OK;
    case SF_OPT_FIT_PACK:
      ctx->fit_pack = value != 0;
      return SF_OK;
    case SF_OPT_FIT_LEAN:
      ctx->fit_lean = value != 0;
      return SF_OK;
    case SF_OPT_EVAL_KS_PAD:
      SF_REQUIRE(value >= 0 && value <= 3, SF_EINVAL,
                 "sf_set_option: k-step padding must be 0..3");
      ctx->eval_ks_pad = value;
      return SF_OK;
    case SF_OPT_EVAL_SLEEP:
      SF_REQUIRE(value >= 0 && value <= 1000, SF_EINVAL,
                 "sf_set_option: eval sleep must be 0..1000");
      ctx->eval_sleep = value;
      return SF_OK;
    case SF_OPT_EVAL_XCD_MAP:
      SF_REQUIRE(value >= -1 && value <= 1, SF_EINVAL,
                 "sf_set_option: XCD map must be -1, 0 or 1");
      ctx->eval_xcd_map = value;
      return SF_OK;
    case SF_OPT_EVAL_GROUPS:
      SF_REQUIRE(value >= 0 && value <= 256 && (value & (value - 1)) == 0,
                 SF_EINVAL, "sf_set_option: groups must be 0 or a power of two <= 256");
      ctx->eval_groups = value;
      return SF_OK;
    case SF_OPT_EVAL_BANDS:
      SF_REQUIRE(value >= 0 && value <= 128 && (value & (value - 1)) == 0,
                 SF_EINVAL, "sf_set_option: bands must be 0 or a power of two <= 128");
      ctx->eval_bands = value;
      return SF_OK;
    case SF_OPT_TESS_SLOTS:
      SF_REQUIRE(value >= 0 && value <= 256, SF_EINVAL,
                 "sf_set_option: tess slots must be 0..256");
      ctx->tess_slots = value;
      return SF_OK;
    case SF_OPT_TESS_TILE:
      SF_REQUIRE(value == 0 || value == 1, SF_EINVAL, "sf_set_option: tess tile must be 0 or 1");
      ctx->tess_tile = value;
      return SF_OK;
    case SF_OPT_TESS_BOX:
      SF_REQUIRE(value >= -1 && value <= 1, SF_EINVAL,
                 "sf_set_option: tess box must be -1, 0 or 1");
      ctx->tess_box = value;
      return SF_OK;
    case SF_OPT_TESS_WAVES:
      SF_REQUIRE(value == 0 || value == 4 || value == 8 || value == 16, SF_EINVAL,
                 "sf_set_option: tess waves must be 0, 4, 8 or 16");
      ctx->tess_waves = value;
      return SF_OK;
    case SF_OPT_EVAL_MAX_BLOCKS:
      SF_REQUIRE(value >= 0, SF_EINVAL, "sf_set_option: negative block cap");
      ctx->eval_max_blocks = value;
      return SF_OK;
    case SF_OPT_EVAL_INT:
      SF_REQUIRE(value == -1 || value == 0, SF_EINVAL,
                 "sf_set_option: eval int must be -1 or 0");
      ctx->eval_int = value;
      return SF_OK;
    case SF_OPT_EVAL_WG_WAVES:
      SF_REQUIRE(value == 0 || value == 4 || value == 8, SF_EINVAL,
                 "sf_set_option: eval workgroup waves must be 0, 4 or 8");
      ctx->eval_wg_waves = value;
      return SF_OK;
    case SF_OPT_FIT_SUBSET_DELETION:
      SF_REQUIRE(value >= 0 && value <= 3, SF_EINVAL,
                 "SF_OPT_FIT_SUBSET_DELETION must be 0, 1, 2 or 3");
      ctx->fit_subset_deletion = (int)value;
      return SF_OK;
    case SF_OPT_FIT_EIG_WAVES:
      SF_REQUIRE(value >= 0 && value <= 4, SF_EINVAL,
                 "sf_set_option: fit eig waves must be 0..4");
      ctx->fit_eig_waves = value;
      return SF_OK;
    default:
      set_error("sf_set_option: unknown option");
      return SF_EINVAL;
  }
}

int sf_get_eval_kernel(sf_ctx* ctx, int gain, unsigned flags, int* kernel) {
  SF_REQUIRE(ctx && kernel, SF_EINVAL, "sf_get_eval_kernel: bad argument");
  SF_REQUIRE(ctx->ksteps > 0, SF_EINVAL,
             "sf_get_eval_kernel: call sf_set_grid first");
  *kernel = sf::pick_eval_kernel(ctx, gain != 0, flags, true);
  return SF_OK;
}

int sf_get_eval_contraction(sf_ctx* ctx, int gain, unsigned flags, int* contraction) {
  SF_REQUIRE(ctx && contraction, SF_EINVAL, "sf_get_eval_contraction: bad argument");
  SF_REQUIRE(ctx->ksteps > 0, SF_EINVAL,
             "sf_get_eval_contraction: call sf_set_grid first");
  *contraction = sf::eval_int_applies(ctx, gain != 0, flags, true)
                     ? SF_EVAL_CONTRACTION_I8_DIGITS
                     : SF_EVAL_CONTRACTION_F64;
  return SF_OK;
}

int sf_synchronize(sf_ctx* ctx) {
  SF_REQUIRE(ctx, SF_EINVAL, "sf_synchronize: NULL context");
  SF_HIP(hipSetDevice(ctx->device));
  SF_HIP(hipStreamSynchronize(ctx->stream));
  return SF_OK;
}

int sf_alloc(sf_ctx* ctx, size_t bytes, void** p) {
  SF_REQUIRE(ctx && p, SF_EINVAL, "sf_alloc: bad argument");
  SF_HIP(hipSetDevice(ctx->device));
  if (hipMalloc(p, bytes) != hipSuccess) {
    set_error("sf_alloc: hipMalloc failed");
    return SF_ENOMEM;
  }
  return SF_OK;
}

int sf_free(sf_ctx* ctx, void* p) {
  SF_REQUIRE(ctx, SF_EINVAL, "sf_free: NULL context");
  SF_HIP(hipSetDevice(ctx->device));
  SF_HIP(hipFree(p));
  return SF_OK;
}

int sf_copy_h2d(sf_ctx* ctx, void* dst, const void* src, size_t bytes) {
  SF_REQUIRE(ctx && (bytes == 0 || (dst && src)), SF_EINVAL,
             "sf_copy_h2d: bad argument");
  SF_HIP(hipSetDevice(ctx->device));
  SF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  SF_HIP(hipStreamSynchronize(ctx->stream));
  return SF_OK;
}

int sf_copy_d2h(sf_ctx* ctx, void* dst, const void* src, size_t bytes) {
  SF_REQUIRE(ctx && (bytes == 0 || (dst && src)), SF_EINVAL,
             "sf_copy_d2h: bad argument");
  SF_HIP(hipSetDevice(ctx->device));
  SF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  SF_HIP(hipStreamSynchronize(ctx->stream));
  return SF_OK;
}

int sf_set_basis(sf_ctx* ctx, const double* pp, int D, double r0,
                 double beta) {
  SF_REQUIRE(ctx && pp, SF_EINVAL, "sf_set_basis: bad argument");
  SF_REQUIRE(D >= 1 && D <= SF_MAX_DIR, SF_EINVAL,
             "sf_set_basis: D out of range [1, SF_MAX_DIR]");
  SF_REQUIRE(r0 > 0.0, SF_EINVAL, "sf_set_basis: r0 must be > 0");
  SF_HIP(hipSetDevice(ctx->device));
  SF_HIP(hipStreamSynchronize(ctx->stream));
  // invalidate basis and grid until the new basis is complete: a failure
  // below must not leave a context whose D points at freed buffers
  ctx->D = 0;
  ctx->nx = ctx->ny = 0;
  ctx->n_pix = 0;
  SF_TRY(dev_alloc(&ctx->d_pp, (size_t)3 * D));
  SF_TRY(dev_alloc(&ctx->d_c, (size_t)D * D));
  SF_TRY(dev_alloc(&ctx->d_pinv, (size_t)D * D));
  SF_TRY(dev_alloc(&ctx->d_u, (size_t)D * D));
  SF_TRY(dev_alloc(&ctx->d_eig, (size_t)64));
  SF_HIP(hipMemcpy(ctx->d_pp, pp, sizeof(double) * 3 * D,
                   hipMemcpyHostToDevice));
  for (int i = 0; i < 3 * D; ++i) ctx->h_pp[i] = pp[i];
  SF_HIP(hipMemset(ctx->d_eig, 0, 64 * sizeof(double)));
  ctx->D = D;
  ctx->r0 = r0;
  ctx->beta = beta;
  int rc = sf::launch_basis(ctx);
  if (rc == SF_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) {
    set_error("sf_set_basis: basis kernel failed");
    rc = SF_EIO;
  }
  if (rc != SF_OK) ctx->D = 0;
  return rc;
}

int sf_get_basis(sf_ctx* ctx, double* c, double* pinv, double* u,
                 double* eig) {
  SF_REQUIRE(ctx && ctx->D > 0, SF_EINVAL, "sf_get_basis: no basis set");
  SF_HIP(hipSetDevice(ctx->device));
  SF_HIP(hipStreamSynchronize(ctx->stream));
  const size_t n = (size_t)ctx->D * ctx->D * sizeof(double);
  if (c) SF_HIP(hipMemcpy(c, ctx->d_c, n, hipMemcpyDeviceToHost));
  if (pinv) SF_HIP(hipMemcpy(pinv, ctx->d_pinv, n, hipMemcpyDeviceToHost));
  if (u) SF_HIP(hipMemcpy(u, ctx->d_u, n, hipMemcpyDeviceToHost));
  if (eig)
    SF_HIP(hipMemcpy(eig, ctx->d_eig, ctx->D * sizeof(double),
                     hipMemcpyDeviceToHost));
  return SF_OK;
}

int sf_kl_fit(sf_ctx* ctx, const double* phase, const float* weight, int T,
              int F, int A, const int* st_order, const sf_fit_params* p,
              double* coef, double* resid, float* w_out, int32_t* order_out) {
  SF_REQUIRE(ctx && ctx->D > 0, SF_EINVAL, "sf_kl_fit: call sf_set_basis first");
  SF_REQUIRE(phase && weight && st_order && p && coef, SF_EINVAL,
             "sf_kl_fit: NULL argument");
  SF_REQUIRE(T >= 1 && F >= 1 && A >= 1, SF_EINVAL,
             "sf_kl_fit: T, F, A must be >= 1");
  SF_REQUIRE((int64_t)F * A <= INT32_MAX / 2, SF_EINVAL,
             "sf_kl_fit: F * A too large");
  SF_REQUIRE(p->screen_type == SF_SCREEN_PHASE || p->screen_type == SF_SCREEN_TEC ||
                 p->screen_type == SF_SCREEN_AMPLITUDE,
             SF_EINVAL, "sf_kl_fit: unsupported screen type");
  SF_REQUIRE(p->niter >= 1 && p->niter <= 64, SF_EINVAL,
             "sf_kl_fit: niter must be in [1, 64]");
  // the mask hash table holds (2 niter + 2) entries per slot in int indices
  SF_REQUIRE((int64_t)T * F * A * (2 * p->niter + 2) < ((int64_t)1 << 30),
             SF_EINVAL,
             "sf_kl_fit: too many slots for one call (split the time axis)");
  SF_REQUIRE(p->ref_ant >= -1 && p->ant_offset >= 0, SF_EINVAL,
             "sf_kl_fit: bad ref_ant / ant_offset");
  {
    const int rl = p->ref_ant - p->ant_offset;
    SF_REQUIRE(p->ref_ant == -1 || p->ref_phase || (rl >= 0 && rl < A),
               SF_EINVAL,
               "sf_kl_fit: reference station not in this shard and no "
               "ref_phase given");
  }
  for (int a = 0; a < A; ++a)
    SF_REQUIRE(st_order[a] >= 0, SF_EINVAL, "sf_kl_fit: negative order");
  SF_HIP(hipSetDevice(ctx->device));
  if (ctx->skip_cap < (size_t)F * A) {
    SF_TRY(dev_alloc(&ctx->d_skip, (size_t)F * A));
    ctx->skip_cap = (size_t)F * A;
  }
  if (ctx->st_order_cap < (size_t)A) {
    SF_TRY(dev_alloc(&ctx->d_st_order, (size_t)A));
    ctx->st_order_cap = (size_t)A;
  }
  SF_HIP(hipMemcpyAsync(ctx->d_st_order, st_order, sizeof(int) * A,
                        hipMemcpyHostToDevice, ctx->stream));
  return sf::launch_fit(ctx, phase, weight, T, F, A, p, coef, resid, w_out,
                        order_out);
}

int sf_get_fit_stats(sf_ctx* ctx, int* n_masks, int* n_general) {
  SF_REQUIRE(ctx, SF_EINVAL, "sf_get_fit_stats: NULL context");
  int c[4] = {0, 0, 0, 0};
  SF_HIP(hipSetDevice(ctx->device));
  SF_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->d_counters)
    SF_HIP(hipMemcpy(c, ctx->d_counters, sizeof(c), hipMemcpyDeviceToHost));
  if (n_masks) *n_masks = c[0];
  if (n_general) *n_general = c[2];
  return SF_OK;
}

int sf_get_fit_pool(sf_ctx* ctx, uint64_t* masks_host, double* entries_host,
                    int max_masks, int* n_masks) {
  SF_REQUIRE(ctx && n_masks && max_masks >= 0, SF_EINVAL, "sf_get_fit_pool: bad argument");
  SF_REQUIRE(max_masks == 0 || (masks_host && entries_host), SF_EINVAL,
             "sf_get_fit_pool: NULL output");
  SF_HIP(hipSetDevice(ctx->device));
  SF_HIP(hipStreamSynchronize(ctx->stream));
  int c0 = 0;
  if (ctx->d_counters)
    SF_HIP(hipMemcpy(&c0, ctx->d_counters, sizeof(int), hipMemcpyDeviceToHost));
  const int n = ctx->pool_D == ctx->D && (size_t)c0 <= ctx->pool_cap ? c0 : 0;
  *n_masks = n;
  const int k = n < max_masks ? n : max_masks;
  if (k > 0) {
    const size_t entry = (size_t)ctx->D * ctx->D + ctx->D;
    SF_HIP(hipMemcpy(masks_host, ctx->d_pool_mask, k * sizeof(uint64_t),
                     hipMemcpyDeviceToHost));
    SF_HIP(hipMemcpy(entries_host, ctx->d_pool, k * entry * sizeof(double),
                     hipMemcpyDeviceToHost));
  }
  return SF_OK;
}

int sf_set_grid(sf_ctx* ctx, const double* x, int nx, const double* y,
                int ny) {
  SF_REQUIRE(ctx && ctx->D > 0, SF_EINVAL, "sf_set_grid: call sf_set_basis first");
  SF_REQUIRE(x && y && nx >= 1 && ny >= 1, SF_EINVAL, "sf_set_grid: bad grid");
  for (int i = 0; i < nx; ++i)
    SF_REQUIRE(std::isfinite(x[i]), SF_EINVAL, "sf_set_grid: non-finite x coordinate");
  for (int j = 0; j < ny; ++j)
    SF_REQUIRE(std::isfinite(y[j]), SF_EINVAL, "sf_set_grid: non-finite y coordinate");
  SF_REQUIRE((int64_t)nx * ny <= ((int64_t)1 << 31), SF_EINVAL,
             "sf_set_grid: grid too large");
  SF_HIP(hipSetDevice(ctx->device));
  ctx->n_pix = 0;  // no usable grid until the pixel basis is built
  ctx->nx = nx;
  ctx->ny = ny;
  const int64_t n_pix = (int64_t)nx * ny;
  ctx->n_pix_blocks = (n_pix + sf::kBlockPix - 1) / sf::kBlockPix;
  ctx->ksteps = (ctx->D + 3) / 4;
  const size_t n = (size_t)ctx->n_pix_blocks * sf::kEvalWaves * ctx->ksteps *
                   sf::kTiles * 64;
  SF_TRY(dev_alloc(&ctx->d_cfrag, n));
  double* dx = nullptr;
  double* dy = nullptr;
  SF_TRY(dev_alloc(&dx, (size_t)nx));
  int rc = dev_alloc(&dy, (size_t)ny);
  if (rc != SF_OK) {
    hipFree(dx);
    return rc;
  }
  if (hipMemcpyAsync(dx, x, sizeof(double) * nx, hipMemcpyHostToDevice,
                     ctx->stream) != hipSuccess ||
      hipMemcpyAsync(dy, y, sizeof(double) * ny, hipMemcpyHostToDevice,
                     ctx->stream) != hipSuccess) {
    set_error("sf_set_grid: copy of the grid coordinates failed");
    rc = SF_EIO;
  } else {
    rc = sf::launch_cpix(ctx, dx, dy);
  }
  // largest |Cpix| over the grid: |Cpix| = (d^2 / r0^2)^(beta / 2) / 2 is
  // monotonic in the distance, so its maximum is at the farthest grid point
  // of each direction (beta > 0) or at the nearest one (beta < 0); both are
  // taken, with 1 % margin for the device pow.  The fixed-point phase
  // epilogue's group bound and the integer contraction's range check.  A
  // non-finite value (beta < 0 on a piercepoint) disables both.
  double cmax = 0.0;
  for (int d = 0; d < ctx->D; ++d) {
    const double px = ctx->h_pp[3 * d], py = ctx->h_pp[3 * d + 1];
    double mx = 0.0, my = 0.0, nxd = HUGE_VAL, nyd = HUGE_VAL;
    for (int i = 0; i < nx; ++i) {
      mx = std::fmax(mx, std::fabs(px - x[i]));
      nxd = std::fmin(nxd, std::fabs(px - x[i]));
    }
    for (int j = 0; j < ny; ++j) {
      my = std::fmax(my, std::fabs(py - y[j]));
      nyd = std::fmin(nyd, std::fabs(py - y[j]));
    }
    const double z = ctx->h_pp[3 * d + 2];
    for (const double d2 : {mx * mx + my * my + z * z, nxd * nxd + nyd * nyd + z * z}) {
      const double c = 1.01 * 0.5 * std::pow(d2 / (ctx->r0 * ctx->r0), ctx->beta / 2.0);
      cmax = std::isfinite(c) ? std::fmax(cmax, c) : HUGE_VAL;
    }
  }
  // the integer-digit contraction (D >= 45): rint(Cpix * 2^36) must fit 6
  // balanced base-256 digits (|.| < 2^46.99); 2^46.9 leaves the margin, and
  // kl_cdig_kernel reports any value that still does not fit
  ctx->dig_ok = 0;
  int* dbad = nullptr;
  if (rc == SF_OK && ctx->ksteps >= 12 && std::isfinite(cmax) &&
      cmax * 68719476736.0 < std::ldexp(1.0, 46) * 1.86) {
    // (no memory for the digits: the fp64 contraction serves, not an error)
    if (dev_alloc(&ctx->d_cdig, (size_t)ctx->n_pix_blocks * sf::kEvalWaves *
                                    sf::kDigits * sf::kTiles * 64 * 16) == SF_OK &&
        dev_alloc(&dbad, 1) == SF_OK &&
        hipMemsetAsync(dbad, 0, sizeof(int), ctx->stream) == hipSuccess) {
      rc = sf::launch_cdig(ctx, dx, dy, dbad);
      if (rc == SF_OK) ctx->dig_ok = 1;
    }
  }
  if (hipStreamSynchronize(ctx->stream) != hipSuccess && rc == SF_OK) {
    set_error("sf_set_grid: pixel basis kernel failed");
    rc = SF_EIO;
  }
  if (ctx->dig_ok) {
    int bad = 1;
    if (hipMemcpy(&bad, dbad, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess || bad)
      ctx->dig_ok = 0;
  }
  (void)hipFree(dbad);
  (void)hipFree(dx);
  (void)hipFree(dy);
  if (rc == SF_OK) {
    // per lane (a quarter of a slot's directions): 2^17 / 4 turns
    ctx->rev_thr = cmax > 0.0 && std::isfinite(cmax) ? 32768.0 / cmax : 0.0;
    ctx->n_pix = n_pix;
  } else {
    ctx->dig_ok = 0;
  }
  return rc;
}

int sf_kl_eval(sf_ctx* ctx, const double* coef, int64_t S, float* out,
               int64_t ring, unsigned flags) {
  SF_REQUIRE(ctx && ctx->n_pix > 0 && ctx->d_cfrag, SF_EINVAL,
             "sf_kl_eval: call sf_set_grid first");
  SF_REQUIRE(coef && out && S >= 0 && ring >= 1, SF_EINVAL,
             "sf_kl_eval: bad argument");
  if (S == 0) return SF_OK;
  SF_HIP(hipSetDevice(ctx->device));
  return sf::launch_eval(ctx, coef, nullptr, nullptr, S, out, ring, flags,
                         nullptr);
}

int sf_kl_eval_gain(sf_ctx* ctx, const double* coef_phase,
                    const double* coef_xx, const double* coef_yy, int64_t S,
                    float* out, int64_t ring, unsigned flags) {
  SF_REQUIRE(ctx && ctx->n_pix > 0 && ctx->d_cfrag, SF_EINVAL,
             "sf_kl_eval_gain: call sf_set_grid first");
  SF_REQUIRE(coef_phase && coef_xx && coef_yy && out && S >= 0 && ring >= 1,
             SF_EINVAL, "sf_kl_eval_gain: bad argument");
  if (S == 0) return SF_OK;
  SF_HIP(hipSetDevice(ctx->device));
  return sf::launch_eval(ctx, coef_phase, coef_xx, coef_yy, S, out, ring, flags,
                         nullptr);
}

int sf_kl_eval_sums(sf_ctx* ctx, const double* coef_phase,
                    const double* coef_xx, const double* coef_yy, int64_t S,
                    float* out, int64_t ring, unsigned flags,
                    uint32_t* slot_sums) {
  SF_REQUIRE(ctx && ctx->n_pix > 0 && ctx->d_cfrag, SF_EINVAL,
             "sf_kl_eval_sums: call sf_set_grid first");
  SF_REQUIRE(coef_phase && out && slot_sums && S >= 0 && ring >= 1,
             SF_EINVAL, "sf_kl_eval_sums: bad argument");
  SF_REQUIRE((coef_xx == nullptr) == (coef_yy == nullptr), SF_EINVAL,
             "sf_kl_eval_sums: give both amplitude coefficient sets or neither");
  if (S == 0) return SF_OK;
  SF_HIP(hipSetDevice(ctx->device));
  return sf::launch_eval(ctx, coef_phase, coef_xx, coef_yy, S, out, ring, flags,
                         reinterpret_cast<unsigned*>(slot_sums));
}

// scipy.ndimage._gaussian_kernel1d(sigma, 0, int(4 sigma + 0.5)) uploaded to
// ctx->d_gw; R = 0 for sigma <= 1e-15 (the one weight 1.0).  The weights of
// the last sigma stay on the device: repeated calls with the same sigma (every
// chunk of a Screen.write) upload nothing and stay fully asynchronous.
static int upload_gaussian(sf_ctx* ctx, double sigma, int* R_out) {
  if (sigma <= 1e-15) sigma = 0.0;
  const int R = sigma > 0.0 ? (int)(4.0 * sigma + 0.5) : 0;
  *R_out = R;
  if (ctx->d_gw && sigma == ctx->gw_sigma) return SF_OK;
  std::vector<double> w(1, 1.0);
  if (sigma > 0.0) {
    w.assign(2 * R + 1, 0.0);
    double sum = 0.0;
    for (int i = -R; i <= R; ++i)
      w[i + R] = std::exp(-0.5 / (sigma * sigma) * (double)(i * i));
    for (int i = 0; i < 2 * R + 1; ++i) sum += w[i];
    for (int i = 0; i < 2 * R + 1; ++i) w[i] /= sum;
  }
  // new weights (a change of sigma, rare): launches on ANY stream may still
  // read the previous ones, and the host vector dies here -- drain the
  // device, copy on the context's stream, wait for the copy
  SF_HIP(hipDeviceSynchronize());
  // until the copy below has landed d_gw holds no sigma's weights: a failure
  // on the way must not leave the cache naming the old sigma
  ctx->gw_sigma = -1.0;
  if (ctx->gw_cap < w.size()) {
    if (ctx->d_gw) (void)hipFree(ctx->d_gw);
    ctx->d_gw = nullptr;
    ctx->gw_cap = 0;
    const size_t cap = w.size() < 64 ? 64 : w.size();
    if (hipMalloc(reinterpret_cast<void**>(&ctx->d_gw), cap * sizeof(double)) !=
        hipSuccess) {
      set_error("hipMalloc failed");
      return SF_ENOMEM;
    }
    ctx->gw_cap = cap;
  }
  SF_HIP(hipMemcpyAsync(ctx->d_gw, w.data(), w.size() * sizeof(double),
                        hipMemcpyHostToDevice, ctx->stream));
  SF_HIP(hipStreamSynchronize(ctx->stream));
  ctx->gw_sigma = sigma;
  return SF_OK;
}

int sf_tess_fill(sf_ctx* ctx, const int32_t* labels, int nx, int ny,
                 const double* phase, const double* amp_xx,
                 const double* amp_yy, int D, int64_t S, float* out,
                 int64_t ring, double smooth_pix, unsigned flags) {
  SF_REQUIRE(ctx && labels && phase && out, SF_EINVAL, "sf_tess_fill: NULL argument");
  SF_REQUIRE(nx >= 1 && ny >= 1 && D >= 1 && D <= 64 && S >= 0 && ring >= 1 &&
                 ring <= INT32_MAX,
             SF_EINVAL, "sf_tess_fill: bad shape");
  SF_REQUIRE(smooth_pix >= 0.0 && smooth_pix <= 1e4, SF_EINVAL,
             "sf_tess_fill: smooth_pix must be in [0, 1e4]");
  if (S == 0) return SF_OK;
  SF_HIP(hipSetDevice(ctx->device));
  int R = 0;
  int rc = upload_gaussian(ctx, smooth_pix, &R);
  if (rc != SF_OK) return rc;
  if (R <= sf::kTessMaxR)
    return (ctx->tess_tile ? sf::launch_tess_tile : sf::launch_tess)(
        ctx, labels, nx, ny, phase, amp_xx, amp_yy, D, S, out, ring, ctx->d_gw, R, flags);
  // wider Gaussians: gather unsmoothed and unscrubbed, then the separable
  // passes of sf_smooth (scrub / byte swap after smoothing, as the
  // reference); every slot needs its own cube for that
  SF_REQUIRE(ring >= S, SF_EINVAL,
             "sf_tess_fill: smooth_pix > 6 needs ring_slots >= S");
  rc = sf::launch_tess(ctx, labels, nx, ny, phase, amp_xx, amp_yy, D, S, out,
                       ring, ctx->d_gw, 0, 0u);
  if (rc != SF_OK) return rc;
  return sf::launch_smooth(ctx, out, nx, ny, S * 4, ctx->d_gw, R, flags);
}

int sf_smooth(sf_ctx* ctx, float* cube, int nx, int ny, int64_t n_img,
              double smooth_pix, unsigned flags) {
  SF_REQUIRE(ctx && cube && nx >= 1 && ny >= 1 && n_img >= 0, SF_EINVAL,
             "sf_smooth: bad argument");
  SF_REQUIRE(n_img % 4 == 0, SF_EINVAL,
             "sf_smooth: n_img must count whole [4][ny][nx] slot cubes");
  SF_REQUIRE(smooth_pix >= 0.0 && smooth_pix <= 1e4, SF_EINVAL,
             "sf_smooth: smooth_pix must be in [0, 1e4]");
  if (n_img == 0) return SF_OK;
  SF_HIP(hipSetDevice(ctx->device));
  int R = 0;
  const int rc = upload_gaussian(ctx, smooth_pix, &R);
  if (rc != SF_OK) return rc;
  return sf::launch_smooth(ctx, cube, nx, ny, n_img, ctx->d_gw, R, flags);
}

}  // extern "C"

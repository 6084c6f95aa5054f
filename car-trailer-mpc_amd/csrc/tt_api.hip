// C-ABI boundary of libttmpc.so (declared in include/ttmpc.h).
//
// Host side of the drop-in: validates shapes before any launch (a mis-sized LDS or grid is a
// GPU fault), owns per-handle device workspaces for the host-pointer entry point, and forwards
// device-pointer calls straight to the kernel on the caller's stream.  No CPU fallback exists:
// every solve runs the gfx950 kernel in tt_track.hip.
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <thread>
#include <chrono>
#include <atomic>

#include "tt_kernel.hpp"
#include "ttmpc.h"

namespace {

struct Handle {
    tt_config cfg;
    double Q[36], R[4], xlb[6], xub[6], ulb[2], uub[2];
    double obs[4 * ttmpc::kObcaMaxM] = {};
    // OBCA variants: per-instance solver workspace + host-call staging buffers
    size_t ocap = 0;
    double* d_ows = nullptr;
    double *d_oxg = nullptr, *d_ozg = nullptr, *d_ozo = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;
    size_t cap = 0;  // instances the workspace holds
    double *d_x0 = nullptr, *d_xref = nullptr, *d_uref = nullptr, *d_w = nullptr, *d_zg = nullptr;
    double *d_xo = nullptr, *d_uo = nullptr, *d_kkt = nullptr;
    int *d_st = nullptr, *d_it = nullptr;
    // tracking host calls: one packed device input / output block and its pinned host mirror, so a
    // host-pointer solve is one H2D, the launch and one D2H (bytes).  The mirror is coherent (fine-grained) pinned
    // memory: small batches skip both copies and let the kernel read and write it in place (zd_*: its device view)
    size_t stage_in = 0, stage_out = 0;
    char *d_sin = nullptr, *d_sout = nullptr, *h_sin = nullptr, *h_sout = nullptr, *zd_sin = nullptr, *zd_sout = nullptr;
    std::string err;
    unsigned long long* obca_stamps = nullptr;  // diagnostics: per-phase clocks (ttx_obca_set_stamps)
    unsigned long long* d_board = nullptr;      // OBCA helper-workgroup board, (ocap + 1) lines
    int nhelp = -1;                             // OBCA helper workgroups per launch (-1: one per CU; ttx_obca_set_helpers)
    unsigned long long spin_ticks = 0;          // hand-off spin limit (0: 5 s) and forced-timeout instance (-1: none),
    int fail_b = -1;                            //   ttx_obca_set_handoff_debug
    // tracking builds that keep stage rows in HBM (the N = 50 build, ttmpc::track_global_bytes): one launch's rows
    double* d_prow = nullptr;
    size_t prow_cap = 0;  // bytes
};

thread_local std::string g_err;

// Makes the handle's device current for one entry point and restores the caller's device on every
// return path (the C ABI must not leave a different current device behind).
struct DeviceGuard {
    int prev = -1;
    hipError_t err;
    explicit DeviceGuard(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev == device) {
            prev = -1;  // already current: nothing to switch or restore (a B = 1 call pays neither)
            err = hipSuccess;
        } else {
            err = hipSetDevice(device);
        }
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int fail(Handle* h, int code, const char* fmt, const char* detail = "") {
    char buf[512];
    snprintf(buf, sizeof buf, fmt, detail);
    if (h) h->err = buf;
    g_err = buf;
    return code;
}

int hip_fail(Handle* h, hipError_t e, const char* where) {
    char buf[512];
    snprintf(buf, sizeof buf, "%s: %s", where, hipGetErrorString(e));
    if (h) h->err = buf;
    g_err = buf;
    return -EIO;
}

void free_ws(Handle* h) {
    double** dp[] = {&h->d_x0, &h->d_xref, &h->d_uref, &h->d_w, &h->d_zg, &h->d_xo, &h->d_uo, &h->d_kkt};
    for (double** p : dp) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    if (h->d_st) (void)hipFree(h->d_st);
    if (h->d_it) (void)hipFree(h->d_it);
    h->d_st = h->d_it = nullptr;
    h->cap = 0;
}

void free_stage(Handle* h) {
    if (h->d_sin) (void)hipFree(h->d_sin);
    if (h->d_sout) (void)hipFree(h->d_sout);
    if (h->h_sin) (void)hipHostFree(h->h_sin);
    if (h->h_sout) (void)hipHostFree(h->h_sout);
    h->d_sin = h->d_sout = h->h_sin = h->h_sout = h->zd_sin = h->zd_sout = nullptr;
    h->stage_in = h->stage_out = 0;
}

int ensure_stage(Handle* h, size_t in_bytes, size_t out_bytes) {
    if (in_bytes <= h->stage_in && out_bytes <= h->stage_out) return 0;
    // a zero-copy call returns once its statuses are written, before its kernel has retired: let it retire first
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    free_stage(h);
    hipError_t e = hipMalloc((void**)&h->d_sin, in_bytes);
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_sout, out_bytes);
    // coherent: the GPU does not cache these pages, so a kernel reading the mirror in place sees this call's inputs
    // (not an L2 copy of the previous call's) and its output stores are in host memory when the stream completes
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable;
    if (e == hipSuccess) e = hipHostMalloc((void**)&h->h_sin, in_bytes, fl);
    if (e == hipSuccess) e = hipHostMalloc((void**)&h->h_sout, out_bytes, fl);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&h->zd_sin, h->h_sin, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&h->zd_sout, h->h_sout, 0);
    if (e != hipSuccess) {
        free_stage(h);
        return fail(h, -ENOMEM, "staging allocation failed (%s bytes)", std::to_string(in_bytes + out_bytes).c_str());
    }
    h->stage_in = in_bytes;
    h->stage_out = out_bytes;
    return 0;
}

// Largest batch a host-pointer tracking solve runs zero-copy (the kernel reads its inputs from and writes its outputs
// to the coherent pinned mirror; no H2D / D2H on the stream).  Only where the kernel reads its inputs once, at load
// (N < 64: the reference window lives in registers, tt_track.hip regref).  TT_ZERO_COPY_MAX overrides (0: off).
int zero_copy_max() {
    static const int v = [] {
        const char* e = getenv("TT_ZERO_COPY_MAX");
        return e ? atoi(e) : 64;
    }();
    return v;
}

// the HBM stage rows of a launch (grown only: a larger batch waits for the device before the old block is freed)
int ensure_prow(Handle* h, size_t bytes) {
    if (bytes <= h->prow_cap) return 0;
    if (h->d_prow) {
        (void)hipDeviceSynchronize();
        (void)hipFree(h->d_prow);
    }
    h->d_prow = nullptr;
    h->prow_cap = 0;
    if (hipMalloc((void**)&h->d_prow, bytes) != hipSuccess) {
        h->d_prow = nullptr;
        return fail(h, -ENOMEM, "stage-row workspace allocation failed (%s bytes)", std::to_string(bytes).c_str());
    }
    h->prow_cap = bytes;
    return 0;
}

// a status value no kernel writes: the zero-copy path's "not finished yet"
constexpr int kStatusPending = -0x40000000;

// Wait until every instance of a zero-copy call has written its status (host memory; the kernel's release orders the
// instance's other outputs before it).  Spins up to 2 ms, then yields to the OS between looks; gives up after 1 s, and
// the caller then waits for the stream (which also reports a fault that kept a status from ever being written).
bool poll_done(volatile int* st, int B) {
    const auto t0 = std::chrono::steady_clock::now();
    for (long long n = 0;; ++n) {
        int i = 0;
        while (i < B && st[i] != kStatusPending) ++i;
        if (i == B) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return true;
        }
        if ((n & 255) == 255) {
            const auto dt = std::chrono::steady_clock::now() - t0;
            if (dt > std::chrono::seconds(1)) return false;
            if (dt > std::chrono::milliseconds(2)) std::this_thread::yield();
        }
    }
}

bool is_obca(const tt_config& c) { return c.variant == TT_VARIANT_TRACK_OBCA || c.variant == TT_VARIANT_OBCA_PLAN; }

void free_ows(Handle* h) {
    double** dp[] = {&h->d_ows, &h->d_oxg, &h->d_ozg, &h->d_ozo};
    for (double** p : dp) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    if (h->d_board) (void)hipFree(h->d_board);
    h->d_board = nullptr;
    h->ocap = 0;
}

// OBCA solver workspace for B instances (HBM: ~1.8 MB per instance at N=200, M=6)
int ensure_ows(Handle* h, int B) {
    if ((size_t)B <= h->ocap) return 0;
    free_ows(h);
    const size_t b = (size_t)B, N = h->cfg.N, M = h->cfg.M, n = ttmpc::obca_n(h->cfg.N, h->cfg.M);
    hipError_t e = hipMalloc((void**)&h->d_ows, b * ttmpc::obca_ws_doubles(h->cfg.N, h->cfg.M) * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_oxg, b * 6 * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_ozg, b * n * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_ozo, b * n * 8);
    if (e == hipSuccess) e = hipMalloc((void**)&h->d_board, (b + 1) * ttmpc::kObcaBoardStride * 8);
    (void)N; (void)M;
    if (e != hipSuccess) {
        free_ows(h);
        return fail(h, -ENOMEM, "OBCA workspace allocation failed for B=%s", std::to_string(B).c_str());
    }
    h->ocap = b;
    return 0;
}

int ensure_ws(Handle* h, int B) {
    if ((size_t)B <= h->cap) return 0;
    free_ws(h);
    const size_t N = h->cfg.N, nz = is_obca(h->cfg) ? ttmpc::obca_n(h->cfg.N, h->cfg.M) : 8 * N + 6;
    const size_t cap = (size_t)B;
    hipError_t e = hipSuccess;
#define ALLOC(p, bytes) \
    if (e == hipSuccess) e = hipMalloc((void**)&(p), (bytes))
    ALLOC(h->d_x0, cap * 6 * 8);
    ALLOC(h->d_xref, cap * (N + 1) * 6 * 8);
    ALLOC(h->d_uref, cap * N * 2 * 8);
    ALLOC(h->d_w, cap * 8 * 8);
    ALLOC(h->d_zg, cap * nz * 8);
    ALLOC(h->d_xo, cap * (N + 1) * 6 * 8);
    ALLOC(h->d_uo, cap * N * 2 * 8);
    ALLOC(h->d_kkt, cap * 8);
    ALLOC(h->d_st, cap * 4);
    ALLOC(h->d_it, cap * 4);
#undef ALLOC
    if (e != hipSuccess) {
        free_ws(h);
        return fail(h, -ENOMEM, "device workspace allocation failed for B=%s", std::to_string(B).c_str());
    }
    h->cap = cap;
    return 0;
}

void defaults(tt_config& c) {
    const bool relaxed = c.variant == TT_VARIANT_NMPC || c.variant == TT_VARIANT_FUZZY;
    // IPOPT options of the reference classes: mpc_control.py:35-39 (defaults tol 1e-8, acceptable
    // 1e-6 x 15), mpc_control_nmpc.py:36-45 / mpc_control_fuzzy.py:47-58 (tol 1e-3, acc 1e-2 x 5),
    // mpc_control_obs.py:189-193 / trajectory_optimization.py:196-199 (max_iter 5000, IPOPT defaults)
    if (c.tol <= 0) c.tol = relaxed ? 1e-3 : 1e-8;
    if (c.acc_tol <= 0) c.acc_tol = relaxed ? 1e-2 : 1e-6;
    if (c.max_iter <= 0) c.max_iter = relaxed ? 2000 : 5000;
    if (c.acc_iter <= 0) c.acc_iter = relaxed ? 5 : 15;
}

ttmpc::TrackArgs make_args(const Handle* h, int B) {
    ttmpc::TrackArgs a;
    memset(&a, 0, sizeof a);
    a.N = h->cfg.N;
    a.B = B;
    a.max_iter = h->cfg.max_iter;
    a.acc_iter = h->cfg.acc_iter;
    a.dt = h->cfg.dt;
    a.L1 = h->cfg.L1;
    a.L2 = h->cfg.L2;
    a.Mh = h->cfg.Mh;
    a.tol = h->cfg.tol;
    a.acc_tol = h->cfg.acc_tol;
    memcpy(a.Q, h->Q, sizeof a.Q);
    memcpy(a.R, h->R, sizeof a.R);
    memcpy(a.xlb, h->xlb, sizeof a.xlb);
    memcpy(a.xub, h->xub, sizeof a.xub);
    memcpy(a.ulb, h->ulb, sizeof a.ulb);
    memcpy(a.uub, h->uub, sizeof a.uub);
    return a;
}

}  // namespace

extern "C" {

int tt_create(const tt_config* cfg, const double* Q, const double* R, const double* xlb, const double* xub,
              const double* ulb, const double* uub, const double* obstacles, int device, void** handle) {
    if (!handle) return fail(nullptr, -EINVAL, "handle pointer is NULL%s");
    *handle = nullptr;
    if (!cfg || !Q || !R || !xlb || !xub || !ulb || !uub) return fail(nullptr, -EINVAL, "NULL argument%s");
    if (cfg->nx != 6 || cfg->nu != 2)
        return fail(nullptr, -EINVAL, "truck-trailer model has nx=6, nu=2 (truck_trailer_model.py:4-5)%s");
    const bool obca = is_obca(*cfg);
    if (!obca && cfg->variant != TT_VARIANT_TRACK && cfg->variant != TT_VARIANT_NMPC && cfg->variant != TT_VARIANT_FUZZY)
        return fail(nullptr, -EINVAL, "unknown variant%s");
    if (obca) {
        // mpc_control_obs.py:149 / trajectory_optimization.py:25-26 need at least one obstacle
        if (cfg->M < 1 || cfg->M > ttmpc::kObcaMaxM)
            return fail(nullptr, -EINVAL, "OBCA variants need 1 <= M <= %s obstacles",
                        std::to_string(ttmpc::kObcaMaxM).c_str());
        if (!obstacles) return fail(nullptr, -EINVAL, "OBCA variants need the obstacle list (M x [cx, cy, w, h])%s");
        if (cfg->N < 1 || cfg->N > 100000) return fail(nullptr, -EINVAL, "horizon must be in [1, 100000]%s");
        if (!(cfg->W1 > 0) || !(cfg->W2 > 0)) return fail(nullptr, -EINVAL, "params W1, W2 must be > 0%s");
        for (int i = 0; i < 4 * cfg->M; ++i)
            if (!isfinite(obstacles[i])) return fail(nullptr, -EINVAL, "non-finite obstacle entry%s");
    } else if (cfg->N < 1 || cfg->N > ttmpc::max_horizon()) {
        return fail(nullptr, -EINVAL, "horizon must be in [1, %s] (LDS-resident instance)",
                    std::to_string(ttmpc::max_horizon()).c_str());
    }
    if (!(cfg->dt > 0) || !(cfg->L1 > 0) || !(cfg->L2 > 0) || !isfinite(cfg->Mh))
        return fail(nullptr, -EINVAL, "params dt, L1, L2 must be > 0 and M finite%s");
    for (int i = 0; i < 6; ++i)
        if (!(xlb[i] <= xub[i])) return fail(nullptr, -EINVAL, "state bound lb > ub%s");
    for (int i = 0; i < 2; ++i)
        if (!(ulb[i] <= uub[i])) return fail(nullptr, -EINVAL, "input bound lb > ub%s");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(nullptr, -ENODEV, "no HIP device: ttmpc is GPU-only (gfx950)%s");
    if (device < 0 || device >= ndev) return fail(nullptr, -ENODEV, "device ordinal out of range%s");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(nullptr, -ENODEV, "device is not gfx950 (MI355X): %s", prop.gcnArchName);
    Handle* h = new Handle();
    h->cfg = *cfg;
    defaults(h->cfg);
    memcpy(h->Q, Q, sizeof h->Q);
    memcpy(h->R, R, sizeof h->R);
    memcpy(h->xlb, xlb, sizeof h->xlb);
    memcpy(h->xub, xub, sizeof h->xub);
    memcpy(h->ulb, ulb, sizeof h->ulb);
    memcpy(h->uub, uub, sizeof h->uub);
    if (obca) memcpy(h->obs, obstacles, sizeof(double) * 4 * cfg->M);
    h->device = device;
    DeviceGuard dg(device);
    hipError_t e = dg.err;
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        int rc = hip_fail(nullptr, e, "tt_create");
        delete h;
        return rc;
    }
    *handle = h;
    return 0;
}

namespace {
int solve_device_impl(Handle* h, int B, const double* d_x0, const double* d_xref, const double* d_uref,
                      const double* d_wq_wr, const double* d_z_guess, double* d_x_out, double* d_u_out, int* d_status,
                      int* d_iters, double* d_kkt_res, void* stream, int host_done);
}  // namespace

int tt_solve_batch_device(void* handle, int B, const double* d_x0, const double* d_xref, const double* d_uref,
                          const double* d_wq_wr, const double* d_z_guess, double* d_x_out, double* d_u_out,
                          int* d_status, int* d_iters, double* d_kkt_res, void* stream) {
    return solve_device_impl(static_cast<Handle*>(handle), B, d_x0, d_xref, d_uref, d_wq_wr, d_z_guess, d_x_out,
                             d_u_out, d_status, d_iters, d_kkt_res, stream, 0);
}

namespace {
int solve_device_impl(Handle* h, int B, const double* d_x0, const double* d_xref, const double* d_uref,
                      const double* d_wq_wr, const double* d_z_guess, double* d_x_out, double* d_u_out, int* d_status,
                      int* d_iters, double* d_kkt_res, void* stream, int host_done) {
    void* handle = h;
    if (!h) return fail(nullptr, -EINVAL, "NULL handle%s");
    if (B < 0) return fail(h, -EINVAL, "B must be >= 0%s");
    if (B == 0) return 0;
    if (B > (1 << 30)) return fail(h, -EINVAL, "B too large%s");
    if (!d_x0 || !d_xref || !d_uref || !d_x_out || !d_u_out || !d_status)
        return fail(h, -EINVAL, "NULL device buffer%s");
    if (h->cfg.variant == TT_VARIANT_OBCA_PLAN)
        return fail(h, -EINVAL, "plan handles solve through tt_plan_batch / tt_obca_solve_batch%s");
    if (h->cfg.variant == TT_VARIANT_TRACK_OBCA)
        return tt_obca_solve_batch_device(handle, B, d_x0, nullptr, d_xref, d_uref, d_z_guess, d_x_out, d_u_out,
                                          nullptr, d_status, d_iters, d_kkt_res, stream);
    if (h->cfg.variant == TT_VARIANT_FUZZY && !d_wq_wr)
        return fail(h, -EINVAL, "fuzzy variant needs per-instance weights (mpc_control_fuzzy.py:54-58)%s");
    DeviceGuard dg(h->device);
    hipError_t e = dg.err;
    if (e != hipSuccess) return hip_fail(h, e, "hipSetDevice");
    ttmpc::TrackArgs a = make_args(h, B);
    a.x0 = d_x0;
    a.xref = d_xref;
    a.uref = d_uref;
    a.wqwr = d_wq_wr;
    a.zg = d_z_guess;
    a.xout = d_x_out;
    a.uout = d_u_out;
    a.kkt = d_kkt_res;
    a.status = d_status;
    a.iters = d_iters;
    a.host_done = host_done;
    if (const size_t gb = ttmpc::track_global_bytes(a)) {
        const int rc = ensure_prow(h, gb);
        if (rc) return rc;
        a.prow = h->d_prow;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    e = ttmpc::launch_track(a, s);
    if (e != hipSuccess) return hip_fail(h, e, "track kernel launch");
    return 0;
}
}  // namespace

int tt_solve_batch(void* handle, int B, const double* x0, const double* xref, const double* uref,
                   const double* wq_wr, const double* z_guess, double* x_out, double* u_out, int* status,
                   int* iters, double* kkt_res) {
    Handle* h = static_cast<Handle*>(handle);
    if (!h) return fail(nullptr, -EINVAL, "NULL handle%s");
    if (B < 0) return fail(h, -EINVAL, "B must be >= 0%s");
    if (B == 0) return 0;
    if (!x0 || !xref || !uref || !x_out || !u_out || !status) return fail(h, -EINVAL, "NULL host buffer%s");
    if (h->cfg.variant == TT_VARIANT_OBCA_PLAN)
        return fail(h, -EINVAL, "plan handles solve through tt_plan_batch / tt_obca_solve_batch%s");
    if (is_obca(h->cfg))  // MPC+OBCA handle: its own host path (workspace, z_guess layout)
        return tt_obca_solve_batch(handle, B, x0, nullptr, xref, uref, z_guess, x_out, u_out, nullptr, status, iters,
                                   kkt_res);
    // validate everything tt_solve_batch_device would refuse before the staging buffer is touched
    if (h->cfg.variant == TT_VARIANT_FUZZY && !wq_wr)
        return fail(h, -EINVAL, "fuzzy variant needs per-instance weights (mpc_control_fuzzy.py:54-58)%s");
    if (B > (1 << 30)) return fail(h, -EINVAL, "B too large%s");
    DeviceGuard dg(h->device);
    hipError_t e = dg.err;
    if (e != hipSuccess) return hip_fail(h, e, "hipSetDevice");
    // packed layout, instance-major within each array: in  = x0 | xref | uref | [wq_wr] | [z_guess]
    //                                                   out = X | U | kkt | status, iters (int32)
    const size_t N = h->cfg.N, b = (size_t)B, nz = 8 * N + 6;
    const size_t sizes[5] = {b * 6, b * (N + 1) * 6, b * N * 2, wq_wr ? b * 8 : 0, z_guess ? b * nz : 0};
    const double* srcs[5] = {x0, xref, uref, wq_wr, z_guess};
    size_t in_d = 0;
    for (size_t v : sizes) in_d += v;
    const size_t nxo = b * (N + 1) * 6, nuo = b * N * 2, out_d = nxo + nuo + b + b;  // 2 x int32 per instance = 1 double
    int rc = ensure_stage(h, in_d * 8, out_d * 8);
    if (rc) return rc;
    // zero-copy for small batches (B = 1 latency: the two DMA copies cost more than the kernel's few PCIe reads)
    const bool zc = B <= zero_copy_max() && N < 64;
    double* hin = reinterpret_cast<double*>(h->h_sin);
    const double* dptr[5];
    size_t off = 0;
    for (int a = 0; a < 5; ++a) {
        if (sizes[a]) memcpy(hin + off, srcs[a], sizes[a] * 8);
        dptr[a] = reinterpret_cast<const double*>(zc ? h->zd_sin : h->d_sin) + off;
        off += sizes[a];
    }
    hipStream_t s = h->stream;
    if (!zc) {
        e = hipMemcpyAsync(h->d_sin, h->h_sin, in_d * 8, hipMemcpyHostToDevice, s);
        if (e != hipSuccess) return hip_fail(h, e, "H2D copy");
    }
    double* dxo = reinterpret_cast<double*>(zc ? h->zd_sout : h->d_sout);
    double* duo = dxo + nxo;
    double* dkk = duo + nuo;
    int* dst = reinterpret_cast<int*>(dkk + b);
    int* dit = dst + b;
    // zero-copy: status[] in the host block doubles as the instances' completion flags (the kernel writes each last,
    // behind a system-scope release); a pending sentinel, then a poll of host memory instead of the stream wait
    volatile int* hst = zc ? reinterpret_cast<volatile int*>(h->h_sout + (nxo + nuo + b) * 8) : nullptr;
    if (zc)
        for (int i = 0; i < B; ++i) hst[i] = kStatusPending;
    rc = solve_device_impl(h, B, dptr[0], dptr[1], dptr[2], wq_wr ? dptr[3] : nullptr, z_guess ? dptr[4] : nullptr, dxo,
                           duo, dst, dit, dkk, s, zc ? 1 : 0);
    if (rc) {
        (void)hipStreamSynchronize(s);  // the H2D from the pinned staging buffer may still be in flight
        return rc;
    }
    bool done = false;
    if (zc) done = poll_done(hst, B);
    e = zc ? hipSuccess : hipMemcpyAsync(h->h_sout, h->d_sout, out_d * 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess && !done) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_fail(h, e, "solve");
    const double* ho = reinterpret_cast<const double*>(h->h_sout);
    memcpy(x_out, ho, nxo * 8);
    memcpy(u_out, ho + nxo, nuo * 8);
    if (kkt_res) memcpy(kkt_res, ho + nxo + nuo, b * 8);
    const int* hi = reinterpret_cast<const int*>(ho + nxo + nuo + b);
    memcpy(status, hi, b * 4);
    if (iters) memcpy(iters, hi + b, b * 4);
    return 0;
}

#ifdef TT_STAMPS
// Diagnostic-build-only entry point: per-instance phase cycle sums into d_stamps[B][kNumPhases].
int ttx_solve_stamped(void* handle, int B, const double* d_x0, const double* d_xref, const double* d_uref,
                      double* d_x_out, double* d_u_out, int* d_status, int* d_iters, unsigned long long* d_stamps,
                      void* stream) {
    Handle* h = static_cast<Handle*>(handle);
    if (!h || B <= 0 || !d_stamps) return -EINVAL;
    ttmpc::TrackArgs a = make_args(h, B);
    a.x0 = d_x0;
    a.xref = d_xref;
    a.uref = d_uref;
    a.xout = d_x_out;
    a.uout = d_u_out;
    a.status = d_status;
    a.iters = d_iters;
    a.stamps = d_stamps;
    if (const size_t gb = ttmpc::track_global_bytes(a)) {
        const int rc = ensure_prow(h, gb);
        if (rc) return rc;
        a.prow = h->d_prow;
    }
    hipError_t e = ttmpc::launch_track(a, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : hip_fail(h, e, "stamped launch");
}
#endif

int tt_obca_solve_batch_device(void* handle, int B, const double* d_x0, const double* d_xgoal, const double* d_xref,
                               const double* d_uref, const double* d_z_guess, double* d_x_out, double* d_u_out,
                               double* d_z_out, int* d_status, int* d_iters, double* d_kkt_res, void* stream) {
    return tt_obca_solve_batch_iterate_device(handle, B, d_x0, d_xgoal, d_xref, d_uref, d_z_guess, d_x_out, d_u_out,
                                              d_z_out, d_status, d_iters, d_kkt_res, nullptr, stream);
}

int tt_obca_solve_batch_iterate_device(void* handle, int B, const double* d_x0, const double* d_xgoal,
                                       const double* d_xref, const double* d_uref, const double* d_z_guess,
                                       double* d_x_out, double* d_u_out, double* d_z_out, int* d_status, int* d_iters,
                                       double* d_kkt_res, double* d_iterate_out, void* stream) {
    Handle* h = static_cast<Handle*>(handle);
    if (!h) return fail(nullptr, -EINVAL, "NULL handle%s");
    if (!is_obca(h->cfg)) return fail(h, -EINVAL, "handle is not an OBCA variant%s");
    if (B < 0) return fail(h, -EINVAL, "B must be >= 0%s");
    if (B == 0) return 0;
    if (B > (1 << 24)) return fail(h, -EINVAL, "B too large%s");
    const bool plan = h->cfg.variant == TT_VARIANT_OBCA_PLAN;
    if (!d_x0 || !d_x_out || !d_u_out || !d_status) return fail(h, -EINVAL, "NULL device buffer%s");
    if (plan && !d_xgoal) return fail(h, -EINVAL, "plan variant needs the goal states%s");
    if (!plan && (!d_xref || !d_uref)) return fail(h, -EINVAL, "MPC+OBCA variant needs reference states/inputs%s");
    DeviceGuard dg(h->device);
    hipError_t e = dg.err;
    if (e != hipSuccess) return hip_fail(h, e, "hipSetDevice");
    int rc = ensure_ows(h, B);
    if (rc) return rc;
    ttmpc::ObcaArgs a;
    memset(&a, 0, sizeof a);
    a.N = h->cfg.N;
    a.M = h->cfg.M;
    a.B = B;
    a.mode = plan ? ttmpc::OBCA_PLAN : ttmpc::OBCA_TRACK;
    a.max_iter = h->cfg.max_iter;
    a.acc_iter = h->cfg.acc_iter;
    a.dual_init = h->cfg.dual_init;
    a.dt = h->cfg.dt;
    a.L1 = h->cfg.L1;
    a.L2 = h->cfg.L2;
    a.Mh = h->cfg.Mh;
    a.W1 = h->cfg.W1;
    a.W2 = h->cfg.W2;
    a.tol = h->cfg.tol;
    a.acc_tol = h->cfg.acc_tol;
    a.dmin = 0.2;      // trajectory_optimization.py:95, mpc_control_obs.py:67
    a.eq_tol = 1e-5;   // trajectory_optimization.py:136-139
    a.fin_tol = 1e-2;  // trajectory_optimization.py:172-173
    a.tfac = plan ? 100.0 : 1.0;  // trajectory_optimization.py:180 / mpc_control_obs.py:39
    memcpy(a.Q, h->Q, sizeof a.Q);
    memcpy(a.R, h->R, sizeof a.R);
    memcpy(a.xlb, h->xlb, sizeof a.xlb);
    memcpy(a.xub, h->xub, sizeof a.xub);
    memcpy(a.ulb, h->ulb, sizeof a.ulb);
    memcpy(a.uub, h->uub, sizeof a.uub);
    memcpy(a.obs, h->obs, sizeof a.obs);
    a.x0 = d_x0;
    a.xgoal = d_xgoal;
    a.xref = d_xref;
    a.uref = d_uref;
    a.zg = d_z_guess;
    a.xout = d_x_out;
    a.uout = d_u_out;
    a.zout = d_z_out;
    a.status = d_status;
    a.iters = d_iters;
    a.kkt = d_kkt_res;
    a.itout = d_iterate_out;
    a.ws = h->d_ows;
    a.stamps = h->obca_stamps;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (h->nhelp < 0) {  // one helper workgroup per CU: they run while CUs are idle (the batch's tail)
        int cus = 0;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device);
        if (e != hipSuccess) return hip_fail(h, e, "hipDeviceGetAttribute");
        h->nhelp = cus;
    }
    a.board = h->d_board;
    a.nhelp = h->nhelp;
    a.spin_ticks = h->spin_ticks;
    a.fail_b = h->fail_b;
    e = hipMemsetAsync(h->d_board, 0, ((size_t)B + 1) * ttmpc::kObcaBoardStride * 8, s);
    if (e != hipSuccess) return hip_fail(h, e, "hipMemsetAsync (OBCA board)");
    e = ttmpc::launch_obca(a, s);
    if (e != hipSuccess) return hip_fail(h, e, "OBCA kernel launch");
    return 0;
}

int tt_obca_solve_batch(void* handle, int B, const double* x0, const double* xgoal, const double* xref,
                        const double* uref, const double* z_guess, double* x_out, double* u_out, double* z_out,
                        int* status, int* iters, double* kkt_res) {
    return tt_obca_solve_batch_iterate(handle, B, x0, xgoal, xref, uref, z_guess, x_out, u_out, z_out, status, iters,
                                       kkt_res, nullptr);
}

int tt_obca_solve_batch_iterate(void* handle, int B, const double* x0, const double* xgoal, const double* xref,
                                const double* uref, const double* z_guess, double* x_out, double* u_out, double* z_out,
                                int* status, int* iters, double* kkt_res, double* iterate_out) {
    Handle* h = static_cast<Handle*>(handle);
    if (!h) return fail(nullptr, -EINVAL, "NULL handle%s");
    if (!is_obca(h->cfg)) return fail(h, -EINVAL, "handle is not an OBCA variant%s");
    if (B < 0) return fail(h, -EINVAL, "B must be >= 0%s");
    if (B == 0) return 0;
    const bool plan = h->cfg.variant == TT_VARIANT_OBCA_PLAN;
    if (!x0 || !status || (plan && !xgoal) || (!plan && (!xref || !uref)))
        return fail(h, -EINVAL, "NULL host buffer%s");
    DeviceGuard dg(h->device);
    hipError_t e = dg.err;
    if (e != hipSuccess) return hip_fail(h, e, "hipSetDevice");
    int rc = ensure_ws(h, B);
    if (rc == 0) rc = ensure_ows(h, B);
    if (rc) return rc;
    const size_t N = h->cfg.N, nz = ttmpc::obca_n(h->cfg.N, h->cfg.M), b = (size_t)B;
    hipStream_t s = h->stream;
#define H2D(d, hp, bytes) \
    if (e == hipSuccess) e = hipMemcpyAsync((d), (hp), (bytes), hipMemcpyHostToDevice, s)
#define D2H(hp, d, bytes) \
    if (e == hipSuccess) e = hipMemcpyAsync((hp), (d), (bytes), hipMemcpyDeviceToHost, s)
    H2D(h->d_x0, x0, b * 6 * 8);
    if (plan) H2D(h->d_oxg, xgoal, b * 6 * 8);
    if (!plan) {
        H2D(h->d_xref, xref, b * (N + 1) * 6 * 8);
        H2D(h->d_uref, uref, b * N * 2 * 8);
    }
    if (z_guess) H2D(h->d_ozg, z_guess, b * nz * 8);
    if (e != hipSuccess) return hip_fail(h, e, "H2D copy");
    // the diagnostic iterate export gets a buffer of its own for this call (it is not a hot-path output)
    const size_t it_bytes = b * ttmpc::obca_iterate_len(h->cfg.N, h->cfg.M) * 8;
    double* d_itout = nullptr;
    if (iterate_out) {
        e = hipMalloc((void**)&d_itout, it_bytes);
        if (e != hipSuccess) return fail(h, -ENOMEM, "iterate export allocation failed for B=%s", std::to_string(B).c_str());
    }
    rc = tt_obca_solve_batch_iterate_device(h, B, h->d_x0, plan ? h->d_oxg : nullptr, plan ? nullptr : h->d_xref,
                                            plan ? nullptr : h->d_uref, z_guess ? h->d_ozg : nullptr, h->d_xo, h->d_uo,
                                            z_out ? h->d_ozo : nullptr, h->d_st, h->d_it, h->d_kkt, d_itout, s);
    if (rc) {
        (void)hipStreamSynchronize(s);
        if (d_itout) (void)hipFree(d_itout);
        return rc;
    }
    if (iterate_out) D2H(iterate_out, d_itout, it_bytes);
    if (x_out) D2H(x_out, h->d_xo, b * (N + 1) * 6 * 8);
    if (u_out) D2H(u_out, h->d_uo, b * N * 2 * 8);
    if (z_out) D2H(z_out, h->d_ozo, b * nz * 8);
    D2H(status, h->d_st, b * 4);
    if (iters) D2H(iters, h->d_it, b * 4);
    if (kkt_res) D2H(kkt_res, h->d_kkt, b * 8);
#undef H2D
#undef D2H
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (d_itout) {
        if (e != hipSuccess) (void)hipStreamSynchronize(s);
        (void)hipFree(d_itout);
    }
    if (e != hipSuccess) return hip_fail(h, e, "OBCA solve");
    return 0;
}

/* diagnostics only (not part of include/ttmpc.h): per-instance phase cycle sums of the handle's next OBCA
 * launches into d_stamps[B][kObcaPhases] (device pointer; NULL switches it off).  Returns the phase count. */
int ttx_obca_set_stamps(void* handle, unsigned long long* d_stamps) {
    Handle* h = static_cast<Handle*>(handle);
    if (h) h->obca_stamps = d_stamps;
    return ttmpc::kObcaPhases;
}

/* diagnostics only: helper workgroups of the handle's OBCA launches (0: none, every instance runs its own block
 * passes; -1: one per CU, the default).  The results are bitwise the same either way (tests/test_gpu_obca.py). */
int ttx_obca_set_helpers(void* handle, int n) {
    Handle* h = static_cast<Handle*>(handle);
    if (!h) return -EINVAL;
    h->nhelp = n < 0 ? -1 : n;
    return 0;
}

/* diagnostics only: the helper hand-off's spin limit in microseconds (0: the default 5 s) and one instance whose
 * hand-offs never complete (-1: none), so that it ends with TT_HANDOFF_TIMEOUT while its neighbours solve normally
 * (tests/test_gpu_obca.py::test_helper_handoff_timeout_is_reported_and_isolated). */
int ttx_obca_set_handoff_debug(void* handle, long long spin_us, int fail_b) {
    Handle* h = static_cast<Handle*>(handle);
    if (!h || spin_us < 0) return -EINVAL;
    h->spin_ticks = (unsigned long long)spin_us * 100ull;  // s_memrealtime: 100 MHz
    h->fail_b = fail_b < 0 ? -1 : fail_b;
    return 0;
}
static_assert(TT_HANDOFF_TIMEOUT == 6, "tt_obca.hip kStatusHandoffTimeout");

int tt_plan_batch(void* handle, int B, const double* x0, const double* xgoal, const double* z_guess, double* x_out,
                  double* u_out, int* status, int* iters) {
    Handle* h = static_cast<Handle*>(handle);
    if (!h) return fail(nullptr, -EINVAL, "NULL handle%s");
    if (h->cfg.variant != TT_VARIANT_OBCA_PLAN) return fail(h, -EINVAL, "tt_plan_batch needs a TT_VARIANT_OBCA_PLAN handle%s");
    if (!x_out || !u_out) return fail(h, -EINVAL, "NULL host buffer%s");
    return tt_obca_solve_batch(handle, B, x0, xgoal, nullptr, nullptr, z_guess, x_out, u_out, nullptr, status, iters,
                               nullptr);
}

void tt_destroy(void* handle) {
    Handle* h = static_cast<Handle*>(handle);
    if (!h) return;
    DeviceGuard dg(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    free_ws(h);
    free_ows(h);
    free_stage(h);
    if (h->d_prow) (void)hipFree(h->d_prow);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
}

const char* tt_last_error(void* handle) {
    Handle* h = static_cast<Handle*>(handle);
    return h ? h->err.c_str() : g_err.c_str();
}

int tt_lds_bytes(int N) { return ttmpc::lds_bytes(N); }
int tt_max_horizon(void) { return ttmpc::max_horizon(); }
const char* tt_version(void) { return "ttmpc 0.2 (gfx950: wave-per-instance Riccati IPM; workgroup-per-instance OBCA IPM)"; }
long long tt_obca_n(int N, int M) { return (N < 1 || M < 1) ? -EINVAL : (long long)ttmpc::obca_n(N, M); }
long long tt_obca_iterate_len(int N, int M) {
    return (N < 1 || M < 1) ? -EINVAL : (long long)ttmpc::obca_iterate_len(N, M);
}
long long tt_obca_workspace_bytes(int N, int M) {
    return (N < 1 || M < 1) ? -EINVAL : (long long)(8 * ttmpc::obca_ws_doubles(N, M));
}

}  // extern "C"

// One process per GPU, device memory and hand-off flags shared between the ranks of a node
// (the KS direct schedule under torch.distributed, ks_dist.DirectPeers): IPC handles of the
// ranks' column buffers, a host page mapped into every rank for the sweep counters, and the
// stream-ordered wait / publish launches (ipc_kernels.hip).
#include <hip/hip_runtime.h>

#include <cstring>

#include "aiy_common.hpp"
#include "ks.hpp"

namespace aiy {
int launch_flags_wait(const unsigned long long* flags, unsigned long long mask,
                      unsigned long long v, long long timeout_ticks, unsigned long long* err,
                      hipStream_t st);
int launch_flag_set(unsigned long long* flags, int q, unsigned long long v, hipStream_t st);
}  // namespace aiy

using namespace aiy;

extern "C" {

int aiy_ipc_get_handle(const void* dptr, void* handle, int64_t* offset) {
    if (!dptr || !handle || !offset) return fail(AIY_BAD_ARG, "NULL argument");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    AIY_HIP(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)dptr));
    hipIpcMemHandle_t h;
    AIY_HIP(hipIpcGetMemHandle(&h, (void*)base));
    static_assert(sizeof h == AIY_IPC_HANDLE_BYTES, "IPC handle size");
    memcpy(handle, &h, sizeof h);
    *offset = (int64_t)((const char*)dptr - (const char*)base);
    return AIY_OK;
}

int aiy_ipc_open(const void* handle, int64_t offset, void** dptr) {
    if (!handle || !dptr || offset < 0) return fail(AIY_BAD_ARG, "bad argument");
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof h);
    void* base = nullptr;
    AIY_HIP(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess));
    *dptr = (char*)base + offset;
    return AIY_OK;
}

int aiy_ipc_close(void* dptr, int64_t offset) {
    if (!dptr || offset < 0) return fail(AIY_BAD_ARG, "bad argument");
    AIY_HIP(hipIpcCloseMemHandle((char*)dptr - offset));
    return AIY_OK;
}

int aiy_host_register(void* p, int64_t bytes, void** dptr) {
    if (!p || bytes <= 0 || !dptr) return fail(AIY_BAD_ARG, "bad argument");
    AIY_HIP(hipHostRegister(p, (size_t)bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    AIY_HIP(hipHostGetDevicePointer(dptr, p, 0));
    return AIY_OK;
}

int aiy_host_unregister(void* p) {
    if (!p) return fail(AIY_BAD_ARG, "NULL pointer");
    AIY_HIP(hipHostUnregister(p));
    return AIY_OK;
}

int aiy_flags_wait(const void* flags, uint64_t mask, uint64_t value, double timeout_s, void* err,
                   void* stream) {
    if (!flags || !err || !(timeout_s > 0)) return fail(AIY_BAD_ARG, "bad argument");
    if (!mask) return AIY_OK;
    return launch_flags_wait((const unsigned long long*)flags, mask, value,
                             (long long)(timeout_s * 1e8), (unsigned long long*)err,
                             (hipStream_t)stream);
}

int aiy_flag_set(void* flags, int32_t slot, uint64_t value, void* stream) {
    if (!flags || slot < 0 || slot >= 64) return fail(AIY_BAD_ARG, "bad argument");
    return launch_flag_set((unsigned long long*)flags, slot, value, (hipStream_t)stream);
}

}  // extern "C"

extern "C" {
// nsweeps Jacobi Howard sweeps of the direct schedule in one call (ks_dist.DirectPeers.sweeps):
// sweep i reads parity p = parity ^ (i & 1) and writes parity p ^ 1, after the neighbours in
// `mask` have published n0 + i, and publishes n0 + i + 1 in `slot`.  Staged: the forecast columns
// peers own are read from a local halo, refreshed every sweep from the owners' buffers (device
// pointer arrays src_p[q] -> dst[q], `col_bytes` each, q < ncopy; system-scope loads) by extra
// block rows of the interior launch, so the copies run beside the interior columns; the
// boundary columns sweep in the next launch.  The publish follows a
// system-scope release of the sweep's writes (an event recorded with hipEventReleaseToSystem), so
// a peer's copy after its wait reads this sweep's values from HBM, not from this device's L2.
int ks_dev_direct_sweeps(ks_dev* h, const void* const* tab0, const void* const* tab1,
                         double* V0, double* V1, double* dV0, double* dV1, double* kopt,
                         int32_t parity, int64_t nsweeps, const void* const* src0,
                         const void* const* src1, void* const* dst, int32_t ncopy,
                         int64_t col_bytes, void* flags, int32_t slot, uint64_t mask, uint64_t n0,
                         double timeout_s, void* err, void* stream, void* copy_stream) {
    if (!h || !tab0 || !tab1 || !V0 || !V1 || !dV0 || !dV1 || !kopt || !flags || !err ||
        nsweeps < 0 || (parity & ~1) || ncopy < 0 || (ncopy && (!src0 || !src1 || !dst)) ||
        (ncopy && (!copy_stream || col_bytes <= 0 || col_bytes % 8)))
        return fail(AIY_BAD_ARG, "bad argument");
    const void* const* tab[2] = {tab0, tab1};
    const void* const* src[2] = {src0, src1};
    double* V[2] = {V0, V1};
    double* dV[2] = {dV0, dV1};
    hipStream_t st = (hipStream_t)stream;
    (void)copy_stream;  // (the copies now run inside the interior launch)
    hipEvent_t ev_rel = nullptr;
    int rc = AIY_OK;
    auto done = [&](int r) {
        if (ev_rel) (void)hipEventDestroy(ev_rel);
        return r;
    };
#define DS_TRY(x)                   \
    do {                            \
        rc = (x);                   \
        if (rc != AIY_OK) return done(rc); \
    } while (0)
    {
        const hipError_t e = hipEventCreateWithFlags(&ev_rel, hipEventDisableTiming | hipEventReleaseToSystem);
        if (e != hipSuccess) return fail(AIY_HIP_ERROR, "hipEventCreateWithFlags: %s", hipGetErrorString(e));
    }
    for (int64_t i = 0; i < nsweeps; ++i) {
        const int p = parity ^ (int)(i & 1);
        DS_TRY(aiy_flags_wait(flags, mask, n0 + (uint64_t)i, timeout_s, err, stream));
        DS_TRY(ks_dev_set_columns(h, tab[p]));
        // interior columns + the halo copy rows in one launch, then the boundary columns
        DS_TRY(ks_dev_howard_fused_part_halo(h, 0, V[p], dV[p], kopt, V[p ^ 1], dV[p ^ 1],
                                             ncopy ? src[p] : nullptr, ncopy ? dst : nullptr,
                                             ncopy, stream));
        DS_TRY(ks_dev_howard_fused_part(h, 1, V[p], dV[p], kopt, V[p ^ 1], dV[p ^ 1], stream));
        const hipError_t e = hipEventRecord(ev_rel, st);  // system-scope release before the publish
        if (e != hipSuccess) return done(fail(AIY_HIP_ERROR, "hipEventRecord: %s", hipGetErrorString(e)));
        DS_TRY(aiy_flag_set(flags, slot, n0 + (uint64_t)i + 1, stream));
    }
#undef DS_TRY
    return done(AIY_OK);
}

// the halo refresh alone (before an improvement): the same copies, stream-ordered
int ks_dev_halo_copy(const void* const* src, void* const* dst, int32_t ncopy, int64_t col_bytes,
                     void* stream) {
    if (ncopy < 0 || (ncopy && (!src || !dst || col_bytes <= 0 || col_bytes % 8)))
        return fail(AIY_BAD_ARG, "bad argument");
    return launch_ks_halo_copy(reinterpret_cast<const double* const*>(src),
                               reinterpret_cast<double* const*>(dst), ncopy, (int)(col_bytes / 8),
                               (hipStream_t)stream);
}
}  // extern "C"

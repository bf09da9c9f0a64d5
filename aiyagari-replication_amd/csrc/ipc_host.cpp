// One process per GPU, device memory and hand-off flags shared between the ranks of a node
// (the KS direct schedule under torch.distributed, ks_dist.DirectPeers): IPC handles of the
// ranks' column buffers, a host page mapped into every rank for the sweep counters, the
// stream-ordered wait / publish launches (ipc_kernels.hip) and the staged sweeps, whose waits
// and publishes run inside the sweep launch itself (ks_staged_sweep_kernel).
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
// nsweeps Jacobi Howard sweeps of the direct schedule in one call (ks_dist.DirectPeers.sweeps),
// ONE launch per sweep (ks_dev_staged_sweep) on three buffers per rank: version v lives in
// buffer (v - 1) mod 3, so sweep i reads version n0 + i in buffer b = (cur + i) mod 3 (column
// table tabs[b]) and writes buffer (b + 1) mod 3, which its neighbours last read at version
// n0 + i - 2.  The launch publishes n0 + i (its predecessor's version) first,
// copies the peers' forecast columns of version n0 + i (srcs[b][q] -> dst[q], device pointer
// arrays) once the neighbours in `mask` have published it, sweeps the interior columns without
// waiting and the boundary columns after the copies; a last one-wave launch publishes
// n0 + nsweeps.  tabs, V, dV and srcs are host arrays of three device pointers.
int ks_dev_direct_sweeps(ks_dev* h, void* const* tabs, double* const* V, double* const* dV,
                         double* kopt, int32_t cur, int64_t nsweeps, void* const* srcs,
                         void* const* dst, int32_t ncopy, int64_t col_bytes, void* flags,
                         int32_t slot, uint64_t mask, uint64_t n0, double timeout_s, void* err,
                         void* stream) {
    if (!h || !tabs || !V || !dV || !kopt || !flags || !err || nsweeps < 0 || cur < 0 || cur > 2 ||
        ncopy < 0 || (ncopy && (!srcs || !dst || col_bytes <= 0 || col_bytes % 8)))
        return fail(AIY_BAD_ARG, "bad argument");
    for (int b = 0; b < 3; ++b)
        if (!tabs[b] || !V[b] || !dV[b] || (ncopy && !srcs[b])) return fail(AIY_BAD_ARG, "NULL buffer");
    for (int64_t i = 0; i < nsweeps; ++i) {
        const int b = (int)((cur + i) % 3), bo = (b + 1) % 3;
        const uint64_t v = n0 + (uint64_t)i;
        AIY_TRY(ks_dev_set_columns(h, reinterpret_cast<const void* const*>(tabs[b])));
        AIY_TRY(ks_dev_staged_sweep(h, V[b], dV[b], kopt, V[bo], dV[bo],
                                    ncopy ? reinterpret_cast<const void* const*>(srcs[b]) : nullptr,
                                    ncopy ? dst : nullptr, ncopy, flags, mask, v, slot, v,
                                    timeout_s, err, stream));
    }
    return aiy_flag_set(flags, slot, n0 + (uint64_t)nsweeps, stream);
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

// One process per GPU, device memory and hand-off flags shared between the ranks of a node
// (the KS direct schedule under torch.distributed, ks_dist.DirectPeers): IPC handles of the
// ranks' column buffers, a host page mapped into every rank for the sweep counters, and the
// stream-ordered wait / publish launches (ipc_kernels.hip).
#include <hip/hip_runtime.h>

#include <cstring>

#include "aiy_common.hpp"

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
// sweep i reads parity p = parity ^ (i & 1) through tab[p] and writes parity p ^ 1, after the
// neighbours in `mask` have published n0 + i, and publishes n0 + i + 1 in `slot`
int ks_dev_direct_sweeps(ks_dev* h, const void* const* tab0, const void* const* tab1,
                         double* V0, double* V1, double* dV0, double* dV1, double* kopt,
                         int32_t parity, int64_t nsweeps, void* flags, int32_t slot, uint64_t mask,
                         uint64_t n0, double timeout_s, void* err, void* stream) {
    if (!h || !tab0 || !tab1 || !V0 || !V1 || !dV0 || !dV1 || !kopt || !flags || !err ||
        nsweeps < 0 || (parity & ~1))
        return fail(AIY_BAD_ARG, "bad argument");
    const void* const* tab[2] = {tab0, tab1};
    double* V[2] = {V0, V1};
    double* dV[2] = {dV0, dV1};
    for (int64_t i = 0; i < nsweeps; ++i) {
        const int p = parity ^ (int)(i & 1);
        AIY_TRY(aiy_flags_wait(flags, mask, n0 + (uint64_t)i, timeout_s, err, stream));
        AIY_TRY(ks_dev_set_columns(h, tab[p]));
        AIY_TRY(ks_dev_howard_fused(h, V[p], dV[p], kopt, V[p ^ 1], dV[p ^ 1], stream));
        AIY_TRY(aiy_flag_set(flags, slot, n0 + (uint64_t)i + 1, stream));
    }
    return AIY_OK;
}
}  // extern "C"

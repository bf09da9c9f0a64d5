// Library-owned device buffers of the host tier, cached per (device, shape).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <string>
#include <utility>

#include "../../include/aiyagari_hip.h"

namespace aiy {

struct HostCtx {
    aiy_ws* ws = nullptr;
    hipStream_t st = nullptr;
    std::map<std::string, std::pair<void*, size_t>> bufs;
    int buf(const char* name, size_t bytes, void** out);
    ~HostCtx();
};

int get_ctx(int64_t N, int64_t Na, int64_t Nl, HostCtx** out);
std::mutex& host_mutex();
void cm_to_rows(const double* cm, int64_t N, int64_t Na, double* rows);
void rows_to_cm(const double* rows, int64_t N, int64_t Na, double* cm);
int check_grid(const double* a, int64_t Na);
int check_grid_strict(const double* a, int64_t Na);
int stage_common(HostCtx* c, const double* a, const double* s, const double* P, int64_t N,
                 int64_t Na, double** da, double** ds, double** dP);

}  // namespace aiy

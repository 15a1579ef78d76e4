// Shared by kernarg_probe.hip and kernarg_probe_pre.hip (tools/diag): the probe's grid and argument block.
#pragma once
#include <hip/hip_runtime.h>
constexpr int kBlocks = 2048;
typedef float v4f __attribute__((ext_vector_type(4)));
struct BigArgs {   // ~600 B, the step kernel's argument size; the pointers last
    float pad[148];
    const v4f *in;
    v4f *out;
};
void launch_copy_preload(hipStream_t st, v4f *in, v4f *out);
void launch_copy_big_preload(hipStream_t st, v4f *in, v4f *out);

// Micro-benchmark (diagnostic, not part of the product): ISSUE cost of the instruction kinds in
// the wavefront tick, one wave alone on its SIMD, independent instruction streams (8 chains
// interleaved), measured with clock64 on gfx950.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o ubench_issue scripts/ubench_issue.hip
//   ./ubench_issue
#include <hip/hip_runtime.h>

#include <cstdio>

#define N 128

// 8 independent f64 add chains: cycles per v_add_f64 when issue-bound
__global__ void k_add_f64(double* out, double x, long long* cyc) {
    double a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = x + threadIdx.x + j;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = a[j] + 1.000000001;
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j];
    out[threadIdx.x & 1023] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_mul_f64(double* out, double x, long long* cyc) {
    double a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = x + threadIdx.x + j;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = a[j] * 1.000000001;
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j];
    out[threadIdx.x & 1023] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_add_f32(float* out, float x, long long* cyc) {
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = x + threadIdx.x + j;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) a[j] = a[j] + 1.0001f;
    }
    long long t1 = clock64();
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j];
    out[threadIdx.x & 1023] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// 8 independent 32-bit integer add chains
__global__ void k_add_u32(unsigned* out, unsigned x, long long* cyc) {
    unsigned a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = x + threadIdx.x * 3u + j;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            a[j] = a[j] + (unsigned)(j + 7);
            asm volatile("" : "+v"(a[j]));
        }
    }
    long long t1 = clock64();
    unsigned s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j];
    out[threadIdx.x & 1023] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// f64 selects on a per-lane condition: 8 independent v_cndmask pairs per iteration
__global__ void k_sel_f64(double* out, double x, long long* cyc) {
    double a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = x + threadIdx.x + j;
        b[j] = x - j;
    }
    const bool c = (threadIdx.x & 3) == 1;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            a[j] = c ? b[j] : a[j];
            b[j] = c ? a[j] : b[j];
            asm volatile("" : "+v"(a[j]), "+v"(b[j]));
        }
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += a[j] + b[j];
    out[threadIdx.x & 1023] = s;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// dependent chain: the Muskingum update of one node (4 mul, 4 add, 0 + ...)
__global__ void k_update_chain(double* out, double x, long long* cyc) {
    double o = x + threadIdx.x, I = 1.5, ip = 0.5, q = 0.25;
    const double al = -0.33, be = 0.6, ch = 0.7, ga = 0.3;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) o = 0.0 + (((al * o + be * ip) + ch * I) + ga * q);
    long long t1 = clock64();
    out[threadIdx.x] = o;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <class T, class F>
void run(const char* name, F kern, double per_iter) {
    T* out;
    long long* cyc;
    (void)hipMalloc(&out, 1024 * sizeof(T));
    (void)hipMalloc(&cyc, sizeof(long long));
    for (int threads : {64, 256, 512, 1024}) {   // 1 wave; 1 / 2 / 4 waves per SIMD
        long long h = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(kern, 1, threads, 0, 0, out, (T)1, cyc);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        }
        printf("%-20s %5d threads: %7.2f cycles per instruction per wave\n", name, threads,
               (double)h / (N * per_iter));
    }
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main() {
    run<double>("v_add_f64", k_add_f64, 8);
    run<double>("v_mul_f64", k_mul_f64, 8);
    run<float>("v_add_f32", k_add_f32, 8);
    run<unsigned>("v_add_u32", k_add_u32, 8);
    run<double>("select f64 (2 inst)", k_sel_f64, 32);
    run<double>("update chain/node", k_update_chain, 1);
    return 0;
}

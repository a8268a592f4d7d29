// Micro-benchmark (diagnostic, not part of the product): dependent-latency of the operations on
// the wavefront kernel's critical path, measured with s_memtime on gfx950.
//   hipcc --offload-arch=gfx950 -O3 -o ubench scripts/ubench_latency.hip && ./ubench
#include <hip/hip_runtime.h>

#include <cstdio>

#define N 256

__global__ void k_add_f64(double* out, double x, long long* cyc) {
    double a = x + threadIdx.x;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
        a = a + 1.000000001;
        a = a + 0.999999999;
        a = a + 1.000000001;
        a = a + 0.999999999;
    }
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_mul_f64(double* out, double x, long long* cyc) {
    double a = x + threadIdx.x;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
        a = a * 1.000000001;
        a = a * 0.999999999;
        a = a * 1.000000001;
        a = a * 0.999999999;
    }
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_add_f32(float* out, float x, long long* cyc) {
    float a = x + threadIdx.x;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
        a = a + 1.0001f;
        a = a + 0.9999f;
        a = a + 1.0001f;
        a = a + 0.9999f;
    }
    long long t1 = clock64();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// LDS write -> read of another lane -> write ... (one wave, no barrier)
__global__ void k_lds_chain(double* out, long long* cyc) {
    __shared__ double buf[128];
    const int l = threadIdx.x;
    buf[l] = l;
    __syncthreads();
    double v = 0;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
        v = buf[(l + 1) & 63];
        buf[l] = v + 1.0;
    }
    long long t1 = clock64();
    out[l] = v;
    if (l == 0) cyc[0] = t1 - t0;
}

// barrier chain with B threads (B/64 waves): write, barrier, read neighbour, ...
__global__ void k_barrier_chain(double* out, long long* cyc) {
    __shared__ double buf[2][1024];
    const int l = threadIdx.x;
    buf[0][l] = l;
    __syncthreads();
    double v = 0;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
        v = buf[i & 1][(l + 65) % blockDim.x];
        buf[(i + 1) & 1][l] = v + 1.0;
        __syncthreads();
    }
    long long t1 = clock64();
    out[l] = v;
    if (l == 0) cyc[0] = t1 - t0;
}

// one Muskingum tick without barrier (1 wave): LDS read -> I -> o chain -> LDS write
__global__ void k_tick_chain(double* out, long long* cyc, double al, double be, double ch,
                             double ga) {
    __shared__ double buf[2][128];
    const int l = threadIdx.x;
    buf[0][l] = l;
    buf[1][l] = l;
    __syncthreads();
    double op = 1.0, ip = 2.0, q = 0.5;
    long long t0 = clock64();
#pragma unroll 1
    for (int i = 0; i < N; ++i) {
        const double v0 = buf[i & 1][(l + 1) & 63];
        const double v1 = buf[i & 1][(l + 7) & 63];
        double I = v0 + v1;
        double o = 0.0 + (((al * I + be * ip) + ch * op) + ga * q);
        buf[(i + 1) & 1][l] = o;
        op = o;
        ip = I;
    }
    long long t1 = clock64();
    out[l] = op;
    if (l == 0) cyc[0] = t1 - t0;
}

int main() {
    double* od;
    float* of;
    long long* cy;
    (void)hipMalloc(&od, 1024 * sizeof(double));
    (void)hipMalloc(&of, 1024 * sizeof(float));
    (void)hipMalloc(&cy, 8 * sizeof(long long));
    long long h = 0;
    auto report = [&](const char* name, int ops) {
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(&h, cy, sizeof(h), hipMemcpyDeviceToHost);
        printf("%-28s %8.2f cycles per dependent op\n", name, (double)h / ops);
    };
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_add_f64, 1, 64, 0, 0, od, 1.0, cy);
        report("v_add_f64 (1 wave)", 4 * N);
        hipLaunchKernelGGL(k_mul_f64, 1, 64, 0, 0, od, 1.0, cy);
        report("v_mul_f64 (1 wave)", 4 * N);
        hipLaunchKernelGGL(k_add_f32, 1, 64, 0, 0, of, 1.0f, cy);
        report("v_add_f32 (1 wave)", 4 * N);
        hipLaunchKernelGGL(k_lds_chain, 1, 64, 0, 0, od, cy);
        report("LDS write->read (1 wave)", N);
        for (int b : {64, 128, 256, 512, 1024}) {
            hipLaunchKernelGGL(k_barrier_chain, 1, b, 0, 0, od, cy);
            char name[64];
            snprintf(name, sizeof(name), "barrier tick (%d threads)", b);
            report(name, N);
        }
        hipLaunchKernelGGL(k_tick_chain, 1, 64, 0, 0, od, cy, -0.3, 0.6, 0.7, 0.5);
        report("muskingum tick (1 wave)", N);
    }
    return 0;
}

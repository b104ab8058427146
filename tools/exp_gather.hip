// Gather pricing on MI355X: is a 16-byte gather per lane priced like an
// 8-byte one by the texture addresser (per lane) or twice it (per byte)?
// E = 60M edges, 4 per lane, each naming a vertex inside a 256-vertex block
// that changes every 1,536 edges (the headline edge sweep's v ends within
// its tile runs).  G8: two 8-byte gathers per edge from two arrays (the
// sweep's (X, P) and (Ga, 1/Aux)); G16: one 16-byte gather per edge from
// one interleaved array; S: the same 4 indices per lane and nothing
// gathered (the index stream alone).
//   hipcc -O3 --offload-arch=gfx950 -o exp_gather tools/exp_gather.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void g8(long E, const int4 *__restrict__ idx, const float2 *__restrict__ a,
                   const float2 *__restrict__ b, float *__restrict__ out) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (4 * t >= E) return;
    const int4 i = idx[t];
    const float2 a0 = a[i.x], a1 = a[i.y], a2 = a[i.z], a3 = a[i.w];
    const float2 b0 = b[i.x], b1 = b[i.y], b2 = b[i.z], b3 = b[i.w];
    out[t] = a0.x + a1.y + a2.x + a3.y + b0.x + b1.y + b2.x + b3.y;
}

__global__ void g16(long E, const int4 *__restrict__ idx, const float4 *__restrict__ c,
                    float *__restrict__ out) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (4 * t >= E) return;
    const int4 i = idx[t];
    const float4 c0 = c[i.x], c1 = c[i.y], c2 = c[i.z], c3 = c[i.w];
    out[t] = c0.x + c1.y + c2.z + c3.w + c0.w + c1.z + c2.y + c3.x;
}

__global__ void s0(long E, const int4 *__restrict__ idx, float *__restrict__ out) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (4 * t >= E) return;
    const int4 i = idx[t];
    out[t] = (float)(i.x + i.y + i.z + i.w);
}

int main() {
    const long V = 10000000, E = 60000000;
    std::vector<int> h(E);
    unsigned long long x = 88172645463325252ull;
    for (long e = 0; e < E; e++) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const long base = ((e / 1536) * 256) % (V - 256);
        h[e] = (int)(base + (x & 255));
    }
    int4 *idx; float2 *a, *b; float4 *c; float *out;
    CK(hipMalloc(&idx, E * 4)); CK(hipMalloc(&a, V * 8)); CK(hipMalloc(&b, V * 8));
    CK(hipMalloc(&c, V * 16)); CK(hipMalloc(&out, E));
    CK(hipMemcpy(idx, h.data(), E * 4, hipMemcpyHostToDevice));
    CK(hipMemset(a, 0, V * 8)); CK(hipMemset(b, 0, V * 8)); CK(hipMemset(c, 0, V * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int g = (int)((E / 4 + 255) / 256);
    for (int rep = 0; rep < 3; rep++) {
        for (int k = 0; k < 3; k++) {
            float ms = 0;
            for (int w = 0; w < 2; w++) {  // warm
                if (k == 0) g8<<<g, 256>>>(E, idx, a, b, out);
                else if (k == 1) g16<<<g, 256>>>(E, idx, c, out);
                else s0<<<g, 256>>>(E, idx, out);
            }
            CK(hipEventRecord(e0));
            for (int it = 0; it < 20; it++) {
                if (k == 0) g8<<<g, 256>>>(E, idx, a, b, out);
                else if (k == 1) g16<<<g, 256>>>(E, idx, c, out);
                else s0<<<g, 256>>>(E, idx, out);
            }
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("%s %.4f ms\n", k == 0 ? "G8 (2 x 8 B per edge) " : k == 1 ? "G16 (1 x 16 B per edge)" : "S (indices only)       ",
                   ms / 20);
        }
    }
    return 0;
}

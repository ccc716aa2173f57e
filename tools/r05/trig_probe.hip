// Round 5 diagnostic (not product code): the device's trigonometry against the host C
// library on the inputs the walk kernels feed it. Reads float pairs (y, x) for atan2f and
// angles for sin/cos from a file, writes the device's atan2f, sinf, cosf (OCML), __sinf,
// __cosf (hardware v_sin/v_cos) to another. Usage: trig_probe in.bin out.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void probe(const float* yx, int na, const float* th, int nt, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < na) out[i] = atan2f(yx[2 * i], yx[2 * i + 1]);
    if (i < nt) {
        float t = th[i];
        float* o = out + na + 4 * (size_t)i;
        o[0] = sinf(t); o[1] = cosf(t); o[2] = __sinf(t); o[3] = __cosf(t);
    }
}

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 3;
    int na = 0, nt = 0;
    if (fread(&na, 4, 1, f) != 1 || fread(&nt, 4, 1, f) != 1) return 4;
    std::vector<float> yx(2 * (size_t)na), th(nt), out(na + 4 * (size_t)nt);
    if (fread(yx.data(), 4, yx.size(), f) != yx.size() || fread(th.data(), 4, th.size(), f) != th.size()) return 5;
    fclose(f);
    float *dyx, *dth, *dout;
    if (hipMalloc(&dyx, yx.size() * 4 + 4) || hipMalloc(&dth, th.size() * 4 + 4) || hipMalloc(&dout, out.size() * 4 + 4))
        return 6;
    (void)hipMemcpy(dyx, yx.data(), yx.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dth, th.data(), th.size() * 4, hipMemcpyHostToDevice);
    const int n = na > nt ? na : nt;
    probe<<<(n + 255) / 256, 256>>>(dyx, na, dth, nt, dout);
    if (hipDeviceSynchronize() != hipSuccess) return 7;
    (void)hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
    FILE* g = fopen(argv[2], "wb");
    if (!g) return 8;
    fwrite(out.data(), 4, out.size(), g);
    fclose(g);
    printf("trig_probe: %d atan2, %d angles\n", na, nt);
    return 0;
}

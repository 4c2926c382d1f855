// Probe: can one process IPC-open several allocations from another process
// when their TOTAL exceeds 2 GiB (each allocation alone <= 1 GiB)?
//   ipc_multi_probe 0 <dir> <nbufs> <MiB>   exporter: allocate, publish handles, wait
//   ipc_multi_probe 1 <dir> <nbufs> <MiB>   importer: open each, read a marker
// Build: hipcc --offload-arch=gfx950 -O2 -o ipc_multi_probe ipc_multi_probe.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <vector>

static bool exists(const char* p) { return access(p, F_OK) == 0; }

int main(int argc, char** argv)
{
    if (argc < 5) return 2;
    const int role = atoi(argv[1]);
    const char* dir = argv[2];
    const int nb = atoi(argv[3]);
    const size_t bytes = (size_t)atoll(argv[4]) << 20;
    char hp[512], dp[512];
    snprintf(hp, sizeof(hp), "%s/handles.bin", dir);
    snprintf(dp, sizeof(dp), "%s/done", dir);
    if (role == 0) {
        std::vector<void*> b(nb);
        std::vector<hipIpcMemHandle_t> h(nb);
        for (int i = 0; i < nb; ++i) {
            if (hipMalloc(&b[i], bytes) != hipSuccess) { printf("malloc %d failed\n", i); return 1; }
            int v = 1000 + i;
            (void)hipMemcpy(b[i], &v, 4, hipMemcpyHostToDevice);
            if (hipIpcGetMemHandle(&h[i], b[i]) != hipSuccess) { printf("gethandle %d failed\n", i); return 1; }
        }
        char tmp[520];
        snprintf(tmp, sizeof(tmp), "%s.tmp", hp);
        FILE* f = fopen(tmp, "wb");
        fwrite(h.data(), sizeof(hipIpcMemHandle_t), nb, f);
        fclose(f);
        rename(tmp, hp);
        printf("exporter: %d x %zu MiB published\n", nb, bytes >> 20);
        fflush(stdout);
        for (int t = 0; t < 1200 && !exists(dp); ++t) usleep(50000);
        for (int i = 0; i < nb; ++i) (void)hipFree(b[i]);
        return exists(dp) ? 0 : 1;
    }
    for (int t = 0; t < 1200 && !exists(hp); ++t) usleep(50000);
    std::vector<hipIpcMemHandle_t> h(nb);
    FILE* f = fopen(hp, "rb");
    if (!f || fread(h.data(), sizeof(hipIpcMemHandle_t), nb, f) != (size_t)nb) { printf("no handles\n"); return 1; }
    fclose(f);
    int bad = 0;
    for (int i = 0; i < nb; ++i) {
        void* p = nullptr;
        printf("importer: opening %d (total %zu MiB)...\n", i, ((size_t)(i + 1) * bytes) >> 20);
        fflush(stdout);
        hipError_t e = hipIpcOpenMemHandle(&p, h[i], hipIpcMemLazyEnablePeerAccess);
        int v = -1;
        if (e == hipSuccess) (void)hipMemcpy(&v, p, 4, hipMemcpyDeviceToHost);
        printf("importer: buf %d rc=%d value=%d\n", i, (int)e, v);
        fflush(stdout);
        bad += (e != hipSuccess || v != 1000 + i);
    }
    FILE* d = fopen(dp, "w");
    if (d) fclose(d);
    return bad ? 1 : 0;
}

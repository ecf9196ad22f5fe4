// rt_rccl.cpp — the RCCL gather behind rt_render_gather_async (rt.h
// RT_GATHER_RCCL): one communicator per device of rt_init's list (rank q =
// devs[q], ncclCommInitAll in this process), and the frame's planes gathered
// to rank 0 with ncclGather over xGMI.  This is the collective of SURVEY.md
// §8(e) for a C caller: the reference partitions a frame across pthreads
// (main.c:404-453) or stages it through one device (main_cuda.cu:280-339).
//
// RCCL is loaded on first use (dlopen), not linked: the library is ~0.6 GB
// and only multi-device frames need it.  The copy already in the process (a
// PyTorch-ROCm build's bundled librccl, which matches the HIP runtime that
// process loaded) is preferred; else RT_RCCL_LIB, else librccl.so.1 from the
// ROCm tree (this library's RUNPATH).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <link.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "rt_rccl.h"

namespace rt {
namespace {

struct Rccl {
    bool tried = false;
    void* h = nullptr;
    std::string path, err;
    int version = 0;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) err_str = nullptr;
    decltype(&ncclGetVersion) get_version = nullptr;
};

std::mutex g_rccl_mu;
Rccl g_rccl;
std::vector<int> g_comm_devs;                 // device list the communicators were made for
std::vector<ncclComm_t> g_comms;

int find_loaded(struct dl_phdr_info* info, size_t, void* out)
{
    const char* n = info->dlpi_name;
    if (n && std::strstr(n, "librccl")) {
        *(std::string*)out = n;
        return 1;
    }
    return 0;
}

template <class F>
bool sym(void* h, const char* name, F& f)
{
    f = (F)dlsym(h, name);
    return f != nullptr;
}

// g_rccl_mu held
bool load_locked()
{
    if (g_rccl.tried) return g_rccl.h != nullptr;
    g_rccl.tried = true;
    std::string cand;
    if (const char* e = std::getenv("RT_RCCL_LIB")) cand = e;
    if (cand.empty()) dl_iterate_phdr(find_loaded, &cand);
    if (cand.empty()) cand = "librccl.so.1";
    void* h = dlopen(cand.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        const char* e = dlerror();
        g_rccl.err = std::string("dlopen ") + cand + ": " + (e ? e : "?");
        return false;
    }
    Rccl& r = g_rccl;
    if (!sym(h, "ncclCommInitAll", r.comm_init_all) || !sym(h, "ncclCommDestroy", r.comm_destroy) ||
        !sym(h, "ncclGather", r.gather) || !sym(h, "ncclGroupStart", r.group_start) ||
        !sym(h, "ncclGroupEnd", r.group_end) || !sym(h, "ncclGetErrorString", r.err_str) ||
        !sym(h, "ncclGetVersion", r.get_version)) {
        g_rccl.err = cand + ": missing RCCL symbols (ncclGather needs RCCL, not NCCL)";
        dlclose(h);
        return false;
    }
    r.h = h;
    r.path = cand;
    (void)r.get_version(&r.version);
    return true;
}

std::string nccl_err(const char* what, ncclResult_t e)
{
    return std::string(what) + ": " + (g_rccl.err_str ? g_rccl.err_str(e) : "RCCL error");
}

}  // namespace

int rccl_comms(const std::vector<int>& devs, std::string& err)
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (!load_locked()) {
        err = g_rccl.err;
        return -1;
    }
    if (!g_comms.empty() && g_comm_devs == devs) return 0;
    for (ncclComm_t c : g_comms) (void)g_rccl.comm_destroy(c);
    g_comms.clear();
    g_comm_devs.clear();
    std::vector<ncclComm_t> comms(devs.size());
    int prev = -1;
    (void)hipGetDevice(&prev);
    const ncclResult_t e = g_rccl.comm_init_all(comms.data(), (int)devs.size(), devs.data());
    if (prev >= 0) (void)hipSetDevice(prev);
    if (e != ncclSuccess) {
        err = nccl_err("ncclCommInitAll", e);
        return -1;
    }
    g_comms = comms;
    g_comm_devs = devs;
    return 0;
}

int rccl_gather(const std::vector<int>& devs, const std::vector<const void*>& send, void* recv, size_t count,
                const std::vector<hipStream_t>& streams, std::string& err)
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_comms.empty() || g_comm_devs != devs) {
        err = "RCCL communicators not initialised for this device list";
        return -1;
    }
    int prev = -1;
    (void)hipGetDevice(&prev);
    // one thread drives every rank: the ranks' calls form one group
    ncclResult_t e = g_rccl.group_start();
    for (size_t q = 0; q < devs.size() && e == ncclSuccess; ++q) {
        (void)hipSetDevice(devs[q]);
        e = g_rccl.gather(send[q], q == 0 ? recv : nullptr, count, ncclFloat64, 0, g_comms[q], streams[q]);
    }
    const ncclResult_t e2 = g_rccl.group_end();
    if (prev >= 0) (void)hipSetDevice(prev);
    if (e != ncclSuccess || e2 != ncclSuccess) {
        err = nccl_err("ncclGather", e != ncclSuccess ? e : e2);
        return -1;
    }
    return 0;
}

void rccl_release()
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    for (ncclComm_t c : g_comms) (void)g_rccl.comm_destroy(c);
    g_comms.clear();
    g_comm_devs.clear();
}

std::string rccl_describe()
{
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (!g_rccl.h) return g_rccl.tried ? "rccl unavailable: " + g_rccl.err : "rccl not loaded";
    char buf[64];
    std::snprintf(buf, sizeof buf, "%d.%d.%d", g_rccl.version / 10000, g_rccl.version / 100 % 100,
                  g_rccl.version % 100);
    return std::string("RCCL ") + buf + " (" + g_rccl.path + ")";
}

}  // namespace rt

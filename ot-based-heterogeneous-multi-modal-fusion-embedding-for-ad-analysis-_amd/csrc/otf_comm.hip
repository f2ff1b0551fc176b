// otf_comm.hip — RCCL communicator for the multi-GPU pieces of the path (SURVEY.md §8b
// "otf_comm_* wrappers (RCCL communicator)", §8e): the per-epoch all-gather of the
// embedding shards and the per-iteration all-reduce of the column sums of the
// row-sharded Sinkhorn.  The reference has no collective at all.
//
// RCCL is resolved at run time from the copy already in the process (PyTorch-ROCm
// loads librccl.so.1 for its "nccl" backend), so the library shares one RCCL instance
// with torch.distributed and carries no link-time dependency; a process without it
// loads librccl.so.1 from the ROCm install.  One process per GPU, one rank each.
#include <dlfcn.h>
#include <string.h>

#include "otf_comm.h"

struct otf_comm {
    void* nccl;  // ncclComm_t
    int nranks, rank;
};

namespace otf {
namespace {

using nccl_res = int;
struct Rccl {
    nccl_res (*get_unique_id)(void* id);
    void* comm_init_rank;  // ncclCommInitRank (init_fn below)
    nccl_res (*comm_destroy)(void* comm);
    nccl_res (*all_reduce)(const void* send, void* recv, size_t count, int dtype, int op, void* comm,
                           hipStream_t s);
    nccl_res (*all_gather)(const void* send, void* recv, size_t count, int dtype, void* comm,
                           hipStream_t s);
    bool ok = false;
};

// ncclCommInitRank takes the 128-byte ncclUniqueId BY VALUE: call through an exact
// prototype with that struct type
struct UniqueId {
    char internal[128];
};
using init_fn = nccl_res (*)(void** comm, int nranks, UniqueId id, int rank);

Rccl& rccl() {
    static Rccl r;
    static bool tried = false;
    if (!tried) {
        tried = true;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (h) {
            r.get_unique_id = (nccl_res(*)(void*))dlsym(h, "ncclGetUniqueId");
            r.comm_init_rank = dlsym(h, "ncclCommInitRank");
            r.comm_destroy = (nccl_res(*)(void*))dlsym(h, "ncclCommDestroy");
            r.all_reduce = (nccl_res(*)(const void*, void*, size_t, int, int, void*, hipStream_t))dlsym(
                h, "ncclAllReduce");
            r.all_gather = (nccl_res(*)(const void*, void*, size_t, int, void*, hipStream_t))dlsym(
                h, "ncclAllGather");
            r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_reduce && r.all_gather;
        }
    }
    return r;
}

// otf_dtype -> ncclDataType_t (rccl.h: ncclFloat16 6, ncclFloat32 7, ncclFloat64 8,
// ncclBfloat16 9; bf16: the config-4 encoder outputs, BASELINE.json configs[3])
int nccl_dtype(int32_t dt) {
    switch (dt) {
        case OTF_F32: return 7;
        case OTF_F64: return 8;
        case OTF_F16: return 6;
        case OTF_BF16: return 9;
        default: return -1;
    }
}

}  // namespace

int comm_all_reduce(void* buf, int64_t count, int32_t dtype, int32_t op, otf_comm* comm,
                    hipStream_t s) {
    if (!comm || !buf || count < 0 || (op != OTF_RED_SUM && op != OTF_RED_MAX)) return OTF_EINVAL;
    const int dt = nccl_dtype(dtype);
    if (dt < 0) return OTF_EINVAL;
    if (count == 0) return OTF_OK;
    Rccl& r = rccl();
    if (!r.ok) return OTF_EUNSUPPORTED;
    // rccl.h: ncclSum 0, ncclMax 2
    return r.all_reduce(buf, buf, (size_t)count, dt, op == OTF_RED_SUM ? 0 : 2, comm->nccl, s) == 0
               ? OTF_OK : OTF_EHIP;
}

}  // namespace otf

extern "C" {

int otf_comm_unique_id(void* id_out) {
    if (!id_out) return OTF_EINVAL;
    otf::Rccl& r = otf::rccl();
    if (!r.ok) return OTF_EUNSUPPORTED;
    return r.get_unique_id(id_out) == 0 ? OTF_OK : OTF_EHIP;
}

int otf_comm_init(otf_comm** comm_out, const void* id, int32_t nranks, int32_t rank) {
    if (!comm_out || !id || nranks < 1 || rank < 0 || rank >= nranks) return OTF_EINVAL;
    otf::Rccl& r = otf::rccl();
    if (!r.ok) return OTF_EUNSUPPORTED;
    otf::UniqueId uid;
    memcpy(uid.internal, id, sizeof(uid.internal));
    void* c = nullptr;
    const otf::init_fn init = (otf::init_fn)r.comm_init_rank;
    if (init(&c, nranks, uid, rank) != 0 || !c) return OTF_EHIP;
    otf_comm* h = new otf_comm;
    h->nccl = c;
    h->nranks = nranks;
    h->rank = rank;
    *comm_out = h;
    return OTF_OK;
}

int otf_comm_destroy(otf_comm* comm) {
    if (!comm) return OTF_EINVAL;
    otf::Rccl& r = otf::rccl();
    const int rc = (r.ok && r.comm_destroy(comm->nccl) == 0) ? OTF_OK : OTF_EHIP;
    delete comm;
    return rc;
}

int otf_comm_all_reduce(void* buf, int64_t count, int32_t dtype, int32_t op, otf_comm* comm,
                        otf_stream_t stream) {
    return otf::comm_all_reduce(buf, count, dtype, op, comm, (hipStream_t)stream);
}

int otf_comm_all_gather(const void* send, void* recv, int64_t count_per_rank, int32_t dtype,
                        otf_comm* comm, otf_stream_t stream) {
    if (!comm || !send || !recv || count_per_rank < 0) return OTF_EINVAL;
    const int dt = otf::nccl_dtype(dtype);
    if (dt < 0) return OTF_EINVAL;
    if (count_per_rank == 0) return OTF_OK;
    otf::Rccl& r = otf::rccl();
    if (!r.ok) return OTF_EUNSUPPORTED;
    return r.all_gather(send, recv, (size_t)count_per_rank, dt, comm->nccl, (hipStream_t)stream) == 0
               ? OTF_OK : OTF_EHIP;
}

}  // extern "C"

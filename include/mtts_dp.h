/* Data-parallel gradient exchange for the MI355X training step (libmtts_hip.so, csrc/dp_comm.cpp).
 *
 * The reference trains on one device (train.py:81-84, devices=1); its only collectives are the
 * sync_dist scalar all-reduces of its logging (baselightningmodule.py:117-199).  The north star shards
 * utterances over the GPUs of a node with the gradient all-reduce over RCCL/xGMI overlapped with
 * backward: these entry points replace DDP's bucketed all-reduce (torch/nn/parallel/distributed.py)
 * for the captured training step, where torch's ProcessGroupNCCL cannot be captured on this stack.
 *
 * One communicator per process; ranks and world size are torch.distributed's.  The unique id (128 bytes)
 * is created on rank 0 and broadcast by the caller (any channel, e.g. the torch store).
 * mtts_dp_allreduce_f32 is stream-ordered and may be issued inside HIP stream capture (it becomes
 * graph nodes).  Returns 0 or a negative mtts_status; mtts_last_error() explains.
 */
#ifndef MTTS_DP_H_
#define MTTS_DP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* writes the RCCL unique id (bytes >= 128) */
int mtts_dp_unique_id(void *id_out, size_t bytes);
/* ncclCommInitRank on the caller's current HIP device; *comm_out receives the communicator */
int mtts_dp_comm_init(const void *id, size_t bytes, int32_t nranks, int32_t rank, void **comm_out);
/* in-place all-reduce of count fp32 values: sum, or the mean over ranks when average != 0 */
int mtts_dp_allreduce_f32(void *comm, float *buf, int64_t count, int32_t average, void *hip_stream);
/* the communicator's own view: ranks it spans (ncclCommCount) and this process's rank in it */
int mtts_dp_comm_query(void *comm, int32_t *nranks_out, int32_t *rank_out);
int mtts_dp_comm_destroy(void *comm);
/* the loaded RCCL's version code, -1 if RCCL cannot be loaded */
int mtts_dp_rccl_version(void);

/* Device-side progress for a host watchdog (bench.py's N>1 path): *host_out = nslots int32 in coherent
 * host-mapped memory, zeroed, readable at any time without synchronising the device.
 * mtts_dp_progress_mark is stream-ordered and capturable: tag < 0 adds one to the device's step count and
 * writes it to host[0]; tag >= 0 writes steps * 256 + tag to host[slot] (slot >= 1; the reducer marks
 * bucket k done with tag k + 1 after its all-reduce).  No reference counterpart (the reference has no
 * multi-GPU step; DDP's own watchdog is torch's ProcessGroupNCCL timeout). */
int mtts_dp_progress_create(int32_t nslots, void **handle_out, int32_t **host_out);
int mtts_dp_progress_mark(void *handle, int32_t slot, int32_t tag, void *hip_stream);
int mtts_dp_progress_destroy(void *handle);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* MTTS_DP_H_ */

/*
 * xsknf_gpu.h -- C ABI of the MI355X checksummer batch path.
 *
 * The reference calls one user function per received frame,
 *     int xsknf_packet_processor(void *pkt, unsigned len, unsigned ingress_ifindex);
 * (reference src/xsknf.h:19-23), once per rx descriptor from the per-frame loop of
 * process_batch_1if() (reference src/xsknf.c:654-672).  The checksummer's body is
 * reference examples/checksummer/checksummer_user.c:30-112.
 *
 * This library replaces that per-frame loop with ONE call per rx batch: the
 * whole batch of descriptors is handed over, every frame is checksummed on the
 * GPU, the 2-byte UDP check field is rewritten in place in the UMEM and one
 * verdict per frame is returned, with exactly the reference's meaning:
 *     -1           drop  (frame goes back to the fill ring, src/xsknf.c:663-666)
 *     0..n_if-1    transmit on that interface (tx ring, src/xsknf.c:667-671)
 *
 * Conventions (the reference's own): functions return 0 on success or a
 * negative errno; no torch or HIP types appear in any signature (streams are
 * passed as an opaque `void *` holding a hipStream_t; NULL = default stream).
 */
#ifndef XSKNF_GPU_H
#define XSKNF_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Everything else in the library is hidden (built with -fvisibility=hidden). */
#define XSKNF_GPU_API __attribute__((visibility("default")))

/* Same layout as struct xdp_desc (linux/if_xdp.h), i.e. exactly what the rx
 * ring holds and what xsk_ring_cons__rx_desc() returns (src/xsknf.c:655-656). */
struct xsknf_gpu_desc {
	uint64_t addr;      /* UMEM address; unaligned mode: base | (offset << 48) */
	uint32_t len;       /* frame length in bytes */
	uint32_t options;
};

/* xsk_umem__add_offset_to_addr() (libxdp, used at src/xsknf.c:659) */
#define XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT 48
#define XSKNF_GPU_UNALIGNED_BUF_ADDR_MASK ((1ULL << XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT) - 1)

/* enum action, examples/checksummer/checksummer_user.c:15-18 */
#define XSKNF_CSUM_ACTION_REDIRECT 0
#define XSKNF_CSUM_ACTION_DROP 1

/* The three globals the reference callback reads (checksummer_user.c:24-25,28). */
struct xsknf_csum_opts {
	int32_t csum_iterations;   /* opt_csum_iterations (-i N), default 1; <= 0: no payload sum */
	int32_t action;            /* opt_action (-c REDIRECT|DROP), default REDIRECT */
	uint32_t num_interfaces;   /* config.num_interfaces (must be >= 1 for REDIRECT) */
	uint32_t reserved;         /* must be 0 */
};

/* Library version: (major << 16) | minor. */
XSKNF_GPU_API uint32_t xsknf_gpu_version(void);

/* Number of visible HIP devices in *count. */
XSKNF_GPU_API int xsknf_gpu_device_count(int *count);

/*
 * Checksum one rx batch, asynchronously on `stream`, on the current HIP device.
 * Replaces the loop `for i in batch: verdict[i] = xsknf_packet_processor(pkt_i,
 * len_i, ingress)` of src/xsknf.c:654-672 (pkt_i = umem + translated addr_i).
 *
 *   umem, umem_size   device-resident UMEM (hipMalloc'd, or a device mirror)
 *   descs, n          device-resident rx descriptors (n may be 0)
 *   ingress_ifindex   interface index of the rx socket (0 on the 1-iface path)
 *   opts              host pointer, read before return
 *   verdicts          device array of n int32, written by the kernel
 *   frame_len_hint    largest frame length expected in the batch (0 = 2048);
 *                     a performance hint only: every length is handled correctly
 *   stream            hipStream_t or NULL
 *
 * Descriptors whose [addr, addr+len) lies outside [0, umem_size) are not
 * touched and get verdict -1 (the kernel's own rx validation guarantees the
 * reference never sees one).  The frames of a batch are distinct UMEM chunks,
 * as an rx ring's are (the reference's serial loop would make two descriptors
 * of the same bytes order-dependent; here their frames are checksummed
 * concurrently).
 * A batch runs as one launch per 1M frames (per 16M for frames of at most
 * 128 bytes, where one launch over more frames measured faster; a lane-kernel
 * launch of more than 2M frames loads each lane's window itself and runs 8
 * blocks per CU, the faster shape for a long launch -- for the default shape
 * only: xsknf_gpu_checksum_batch_cfg() with blocks_per_cu != 0 runs exactly
 * the shape it is given).
 * Returns 0, -EINVAL on bad arguments, -EIO on a HIP launch error.
 *
 * Test hook: the environment variable XSKNF_GPU_CU_LIMIT=N sizes every grid as
 * on a device of N CUs (results are unchanged, launches slower; the library
 * says so on stderr once per device).  Not for production use.
 */
XSKNF_GPU_API int xsknf_gpu_checksum_batch(uint8_t *umem, uint64_t umem_size,
		const struct xsknf_gpu_desc *descs, uint32_t n,
		uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts,
		int32_t *verdicts, uint32_t frame_len_hint, void *stream);

/*
 * Launch shape of the batch kernel (tuning / benchmarking).  A group of
 * `lanes_per_frame` lanes (4, 8, 16, 32 or 64) owns one frame at a time and loads
 * `chunks_per_lane` 16-byte chunks per pass; in the register kernel a wave
 * takes tiles of `frames_per_group` consecutive frames per group (the next
 * frame's loads in flight while the current one is reduced); the persistent
 * grid has `blocks_per_cu`
 * 256-thread blocks per CU (0 = 8).  `lds_ring` must be 0 (an LDS-DMA ring
 * kernel, measured slower, was A/B material until round 5; any other value is
 * -EINVAL); `kernel` = XSKNF_GPU_KERNEL_AUTO with lanes_per_frame > 1 selects
 * the register kernel.
 * `lanes_per_frame` = 1 selects the lane kernel for small frames: each lane
 * owns a frame, loads its first `chunks_per_lane` (5..7) chunks itself, and a
 * wave step covers 64 frames (`frames_per_group` = steps per tile); longer
 * frames are finished by a per-lane loop.
 * `fused_stores` = 1 writes every check from the summing kernel itself; 2 parks
 * every check for a second, write-only pass (non-temporal full 64-byte sector
 * rewrites); 0 (default) decides per frame: frames of 1024 bytes or more are
 * deferred (scattered writes mixed into the read stream cost ~25 % of its
 * bandwidth on MI355X), shorter ones write in-line (their check shares the line
 * just read).  3 = records only: the summing kernel runs alone, the UMEM is
 * only read, and every summed frame's verdicts[i] is left as the record
 *   XSKNF_GPU_RECORD_TAG | (u << 16) | check,   u = bits 22..16,
 * meaning "write the 16-bit `check` (as stored in memory, low byte first) at
 * frame offset u + 6, verdict = the forward verdict"; frames that are not
 * summed carry their final verdict.  The STAGED host path uses this mode (the
 * host applies the checks); benchmarks use it to time the summing kernel.
 * In-line checks whose 64-byte sector lies inside the frame are written as
 * that whole sector (group and lane kernels); adding 4 to `fused_stores` writes
 * the 2 check bytes alone instead, adding 8 makes the lane kernel's sector
 * stores plain (write-back) rather than non-temporal (A/B); where the 64 frames
 * of a lane-kernel step lie apart (a 2 KiB-chunk UMEM) its sector stores are
 * written through the L2 (sc1 nt).  Adding 16 (split kernel) patches the
 * deferred checks in the summing kernel itself, once the waves' streams are
 * done, instead of a second launch (the default with 2 for every frame length
 * past the lane kernel's: every check deferred, then patched in bursts at the
 * waves' ends; jumbo frames too since round 5).
 * A frame whose computed check equals the check it already holds (traffic whose
 * UDP checksums a NIC filled in, tests/gen-traffic.lua:120) ends with the bytes
 * it began with (:68 clears the check, :108 stores the same value), so the
 * product kernels write nothing for it and leave its verdict (no record in mode
 * 3).  Adding 32 to `fused_stores` writes such checks anyway (A/B only; the
 * UMEM and verdicts come out the same).
 * `kernel` = XSKNF_GPU_KERNEL_SPLIT selects the split kernel (the default for
 * every hint): lane l of a wave parses, sums and finishes frame l of a
 * 64-frame tile from its first `window_chunks` & 15 (4..7, or 8) chunks, and the
 * payload of longer frames is summed in items of one pass of `lanes_per_frame`
 * x `chunks_per_lane` chunks dealt to the wave's lane groups, `frames_per_group`
 * items per group in flight (any mix of lengths keeps every lane busy);
 * `window_chunks` + 16 loads the windows transposed (W lanes per frame, one
 * coalesced request); + 32 (with + 16, W = 8, 16 x 2 items, two in flight)
 * launches one 12-wave block per CU whose waves draw the CU's tiles from a
 * shared pool (the default up to 4 KiB frames; W = 4, 16 x 3: one 8-wave block
 * per CU, the jumbo default).  Only instantiated shapes are accepted (-EINVAL
 * otherwise); every shape gives identical results.
 */
#define XSKNF_GPU_RECORD_TAG 0x40000000u       /* bits 31..30 = 01 */
#define XSKNF_GPU_RECORD_TAG_MASK 0xC0000000u

#define XSKNF_GPU_KERNEL_AUTO 0    /* group register / lane kernel by the fields above */
#define XSKNF_GPU_KERNEL_SPLIT 1   /* headers by lane, payload by lane groups */

struct xsknf_gpu_launch_cfg {
	int32_t lanes_per_frame;
	int32_t chunks_per_lane;
	int32_t frames_per_group;
	int32_t blocks_per_cu;
	int32_t lds_ring;
	int32_t fused_stores;
	int32_t kernel;          /* XSKNF_GPU_KERNEL_* */
	int32_t window_chunks;   /* split kernel: header window per lane (16-byte chunks), +16 transposed load */
};

/* The shape xsknf_gpu_checksum_batch() uses for a given frame_len_hint. */
XSKNF_GPU_API int xsknf_gpu_default_launch_cfg(uint32_t frame_len_hint, struct xsknf_gpu_launch_cfg *cfg);

/*
 * xsknf_gpu_checksum_batch() for a caller that knows its batch's lengths: the
 * longest frame and the mean length (0 = unknown, as xsknf_gpu_checksum_batch()).
 * The mean picks the shape, which a largest-frame hint alone cannot: up to
 * 4 KiB, one 12-wave block per CU drawing the CU's tiles from a shared pool
 * (1500 B -4 %, 570 B -2 %), except for a mix of mostly short frames (mean
 * < 512 B, e.g. IMIX), which keeps 4-wave blocks and the static schedule
 * (+1.4 % with the pool).  Results are identical whatever the shape.
 */
XSKNF_GPU_API int xsknf_gpu_checksum_batch_lens(uint8_t *umem, uint64_t umem_size,
		const struct xsknf_gpu_desc *descs, uint32_t n,
		uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts,
		int32_t *verdicts, uint32_t frame_len_max, uint32_t frame_len_mean, void *stream);
/* The shape xsknf_gpu_checksum_batch_lens() uses. */
XSKNF_GPU_API int xsknf_gpu_launch_cfg_for_lens(uint32_t frame_len_max, uint32_t frame_len_mean,
		struct xsknf_gpu_launch_cfg *cfg);

/* xsknf_gpu_checksum_batch() with an explicit launch shape instead of a hint. */
XSKNF_GPU_API int xsknf_gpu_checksum_batch_cfg(uint8_t *umem, uint64_t umem_size,
		const struct xsknf_gpu_desc *descs, uint32_t n,
		uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts,
		int32_t *verdicts, const struct xsknf_gpu_launch_cfg *cfg, void *stream);

/*
 * Host-path context: the batch hook as the AF_XDP worker of src/xsknf.c would
 * call it, with the UMEM in host memory (the worker's mmap, src/xsknf.c:958,975)
 * and descriptors / verdicts in host arrays (the rx ring and to_drop / to_tx
 * routing of process_batch_1if, src/xsknf.c:654-672).
 *
 *   XSKNF_GPU_PATH_ZEROCOPY  the UMEM is pinned and mapped; the kernel reads
 *                            the frames and writes the check bytes in place
 *                            over PCIe (no copies).
 *   XSKNF_GPU_PATH_STAGED    only the batch's frame bytes are copied to a device
 *                            mirror (merged runs, or one 2-D copy for frames at
 *                            a constant stride) and checksummed in HBM; only
 *                            the 4-byte records come back and the host writes
 *                            the 2 check bytes.  A batch of frames scattered
 *                            over the UMEM runs as ZEROCOPY instead.
 *   XSKNF_GPU_PATH_RESIDENT  ZEROCOPY without a launch per batch: ONE kernel
 *                            resident on each device serves every RESIDENT
 *                            context of the process on that device (up to 64:
 *                            XSKNF_MAX_WORKERS workers x two UMEMs).  Each
 *                            context has its own ring (the submit writes the
 *                            descriptors and rings a doorbell, the wait spins
 *                            on a completion flag), 8 entries of up to 256
 *                            frames, one block each when max_batch <= 64,
 *                            else four (64 frames each), so up to 8 batches
 *                            per context (or pieces of a larger one) are
 *                            processed at once.  For the rx loop's small
 *                            batches.  The kernel leaves after 1 ms without a
 *                            batch on any ring (and after 4 ms in all) and the
 *                            next submit or wait of any context relaunches it;
 *                            creating or destroying a RESIDENT context stops
 *                            and relaunches it.  It holds one hardware queue
 *                            (GPU_MAX_HW_QUEUES is 4 by default): a process
 *                            that also launches work of its own (ZEROCOPY /
 *                            STAGED contexts, torch) may find a launch queued
 *                            behind it for up to those 4 ms when its streams
 *                            outnumber the hardware queues.  (Measured with 4
 *                            RESIDENT and 4 ZEROCOPY workers in one process:
 *                            no such wait, each side 10-40 % slower per batch
 *                            than alone -- DESIGN 5.3.)  Creating a context returns
 *                            -ENOSPC past 64 rings per device.
 * One context = one worker thread.  A launched context keeps up to five batches in
 * flight (five slots, each with its own HIP stream: four out plus the one being
 * submitted; a deeper hook's submit waits for the oldest): the copies and kernel of
 * one overlap another's, and the host's share of one overlaps the device's share of
 * the others.  A RESIDENT context keeps up to eight (its ring's entries, as many as
 * XSKNF_MAX_HOOK_DEPTH).
 * xsknf_gpu_ctx_process_batch() is synchronous: when it returns, verdicts and
 * check bytes are in host memory (a batch larger than 65536 frames runs as
 * pieces through the slots; if a piece fails to start, the pieces already
 * started are completed before the error returns).  xsknf_gpu_ctx_submit() returns once the batch
 * is enqueued, with a ticket; xsknf_gpu_ctx_wait(ticket) returns once that
 * batch and every earlier one is complete (verdicts written, check bytes in
 * the UMEM).  A submit may itself complete older batches to free a slot.  The
 * frames of batches in flight must not be touched by the caller, and
 * `verdicts` must stay valid, until their wait.
 */
#define XSKNF_GPU_PATH_ZEROCOPY 0
#define XSKNF_GPU_PATH_STAGED 1
#define XSKNF_GPU_PATH_RESIDENT 2

struct xsknf_gpu_ctx;

struct xsknf_gpu_ctx_stats {
	uint64_t batches;
	uint64_t frames;
	uint64_t bytes_h2d;
	uint64_t bytes_d2h;
	uint64_t resident_batches;   /* ring entries the device's resident kernel completed (RESIDENT) */
	uint64_t resident_launches;  /* launches of that kernel so far, for every context of the device */
};

XSKNF_GPU_API int xsknf_gpu_ctx_create(struct xsknf_gpu_ctx **ctx, int device, int path,
		uint32_t max_batch, uint32_t frame_len_hint);
/* Pin (and for ZEROCOPY map) the host UMEM [umem, umem + size). */
XSKNF_GPU_API int xsknf_gpu_ctx_register_umem(struct xsknf_gpu_ctx *ctx, void *umem, uint64_t size);
XSKNF_GPU_API int xsknf_gpu_ctx_process_batch(struct xsknf_gpu_ctx *ctx,
		const struct xsknf_gpu_desc *descs, uint32_t n, uint32_t ingress_ifindex,
		const struct xsknf_csum_opts *opts, int32_t *verdicts);
XSKNF_GPU_API int xsknf_gpu_ctx_submit(struct xsknf_gpu_ctx *ctx, const struct xsknf_gpu_desc *descs,
		uint32_t n, uint32_t ingress_ifindex, const struct xsknf_csum_opts *opts, int32_t *verdicts,
		uint64_t *ticket);
XSKNF_GPU_API int xsknf_gpu_ctx_wait(struct xsknf_gpu_ctx *ctx, uint64_t ticket);
XSKNF_GPU_API int xsknf_gpu_ctx_get_stats(const struct xsknf_gpu_ctx *ctx, struct xsknf_gpu_ctx_stats *stats);
XSKNF_GPU_API int xsknf_gpu_ctx_destroy(struct xsknf_gpu_ctx *ctx);

/* ---- batch hook for the AF_XDP runtime (include/xsknf.h) ------------------
 * The checksummer NF as an xsknf_batch_processor_fn: it replaces the per-frame
 * xsknf_packet_processor() loop of process_batch_1if / process_batch
 * (src/xsknf.c:654-672, :500-522).  Each worker gets its own context (device
 * worker_idx % device count, `path` as above), created on the worker's first
 * batch for each UMEM it sees, so no call crosses threads.  Register with
 *   xsknf_set_batch_processor((xsknf_batch_processor_fn)xsknf_gpu_hook_process, hook);
 * Stop the workers before xsknf_gpu_hook_destroy(), and destroy the hook
 * before xsknf_cleanup() unmaps the UMEMs. */
struct xsknf_gpu_hook;

XSKNF_GPU_API int xsknf_gpu_hook_create(struct xsknf_gpu_hook **hook, const struct xsknf_csum_opts *opts,
		uint32_t workers, int path, uint32_t max_batch, uint32_t frame_len_hint);
XSKNF_GPU_API int xsknf_gpu_hook_process(void *hook, uint32_t worker_idx, void *umem, uint64_t umem_size,
		const struct xsknf_gpu_desc *descs, uint32_t n, uint32_t ingress_ifindex, int32_t *verdicts);
/* The same NF as a two-phase hook (xsknf_batch_submit_fn / xsknf_batch_complete_fn):
 *   xsknf_set_batch_processor_async((xsknf_batch_submit_fn)xsknf_gpu_hook_submit,
 *                                   (xsknf_batch_complete_fn)xsknf_gpu_hook_complete, hook);
 * submit enqueues the batch on the worker's context (xsknf_gpu_ctx_submit),
 * complete waits for its ticket (xsknf_gpu_ctx_wait): the worker receives the
 * next batch while the GPU checksums this one. */
XSKNF_GPU_API int xsknf_gpu_hook_submit(void *hook, uint32_t worker_idx, void *umem, uint64_t umem_size,
		const struct xsknf_gpu_desc *descs, uint32_t n, uint32_t ingress_ifindex, int32_t *verdicts,
		uint64_t *ticket);
XSKNF_GPU_API int xsknf_gpu_hook_complete(void *hook, uint32_t worker_idx, void *umem, uint64_t ticket);
/* Sum of the worker's context stats. */
XSKNF_GPU_API int xsknf_gpu_hook_get_stats(const struct xsknf_gpu_hook *hook, uint32_t worker_idx,
		struct xsknf_gpu_ctx_stats *stats);
XSKNF_GPU_API int xsknf_gpu_hook_destroy(struct xsknf_gpu_hook *hook);

/* ---- one process over several devices (BASELINE config 4) ----------------
 * The reference scales one worker per NIC queue (src/xsknf.c:992, workers
 * started per queue at :1046-1100); frames never cross workers.  The hook above
 * is that model on a node of GPUs (worker w on device w % devices).  These
 * calls are for a global batch that starts on ONE device: it is split into
 * contiguous descriptor ranges balanced by frame bytes, each range's UMEM span
 * and rebased descriptors are moved from the root device to its own by grouped
 * RCCL point-to-point sends over xGMI (one communicator per device,
 * ncclCommInitAll), every device checksums its shard on its own stream, and the
 * counters of all shards are summed by an RCCL all-reduce.  The results equal
 * one device's pass over the whole batch (tests/test_gpu_multi.py). */

/* The byte-balanced split of n descriptors into nshards contiguous ranges:
 * shard k is frames [bounds[k], bounds[k+1]) (bounds: nshards + 1 entries),
 * cut after the first frame whose running sum of lengths reaches
 * total * k / nshards (xsknf_amd/shard.py shard_by_bytes); spans (NULL, or
 * 2 * nshards entries) = each shard's UMEM byte span [lo, hi) over its frames
 * inside [0, umem_size) ({0, 0} for none).  Host arrays; no GPU call. */
XSKNF_GPU_API int xsknf_gpu_shard_plan(const struct xsknf_gpu_desc *descs, uint64_t n, uint64_t umem_size,
		uint32_t nshards, uint64_t *bounds, uint64_t *spans);
/* A shard's descriptors relative to its span's first byte b0 (plain aligned-mode
 * addresses); a descriptor outside [0, umem_size) gets an address past any
 * UMEM (1 << 47): its verdict is -1 and no byte is touched, as before.  Host
 * arrays; no GPU call. */
XSKNF_GPU_API int xsknf_gpu_shard_rebase(const struct xsknf_gpu_desc *descs, uint64_t n, uint64_t b0,
		uint64_t umem_size, struct xsknf_gpu_desc *out);

struct xsknf_gpu_multi;

/* [frames, frame bytes, drops (-1), forwards (>= 0), sum of the 16-bit words at
 * +40 of every frame of >= 42 bytes (an ihl-5 frame's UDP check), the same
 * weighted by ((global UMEM offset) mod 65521) + 1] */
#define XSKNF_GPU_MULTI_COUNTERS 6

#define XSKNF_GPU_SHARD_PACKED 1u   /* shard_info.flags: moved by xsknf_gpu_multi_scatter_packed */

struct xsknf_gpu_shard_info {
	int32_t device;          /* HIP device of the shard */
	uint32_t flags;          /* XSKNF_GPU_SHARD_PACKED */
	uint64_t frame_lo, frame_hi;   /* frames [lo, hi) of the global batch */
	uint64_t span_lo, span_hi;     /* its bytes [lo, hi) of the root's UMEM (packed: 0 and the
	                                  shard's packed bytes) */
	uint64_t frame_bytes;          /* sum of its frame lengths */
	uint8_t *umem;                 /* device buffers of the shard on its device */
	struct xsknf_gpu_desc *descs;
	int32_t *verdicts;
};

/* The packed layout of xsknf_gpu_multi_scatter_packed (no GPU): for shards
 * [bounds[k], bounds[k+1]) of n descriptors over a UMEM at device address
 * umem_addr, each frame gets a 16-byte aligned slot in its shard's packed
 * buffer, at the same address mod 16 as in the UMEM; packed[f] is frame f's
 * descriptor there (its length and options kept; a descriptor outside the
 * UMEM gets an address past any span and no slot), sizes[k] shard k's packed
 * bytes.  A frame of len bytes at address a mod 16 = r takes round16(r + len). */
XSKNF_GPU_API int xsknf_gpu_shard_pack_plan(const struct xsknf_gpu_desc *descs, uint64_t n, uint64_t umem_addr,
		uint64_t umem_size, uint32_t nshards, const uint64_t *bounds, struct xsknf_gpu_desc *packed,
		uint64_t *sizes);
/* One RCCL communicator per device of devices[0..ndev) (NULL: devices 0..ndev-1,
 * each at most once), a stream each. */
XSKNF_GPU_API int xsknf_gpu_multi_create(struct xsknf_gpu_multi **m, const int *devices, int ndev);
/* Split the global batch -- `umem` (umem_size bytes) resident on device
 * devices[root], `descs` its n descriptors in host memory -- by
 * xsknf_gpu_shard_plan and move every shard to its device: one grouped set of
 * ncclSend / ncclRecv, the root's own shard as a send to itself.  Shard buffers
 * are allocated on first use and kept for later scatters of the same size or
 * smaller.  *seconds (may be NULL): wall time of the transfers. */
XSKNF_GPU_API int xsknf_gpu_multi_scatter(struct xsknf_gpu_multi *m, int root, const uint8_t *umem,
		uint64_t umem_size, const struct xsknf_gpu_desc *descs, uint64_t n, double *seconds);
/* Checksum every device's shard (xsknf_gpu_checksum_batch_lens on its own
 * stream, all devices in flight at once); returns when all are done.  ms (may be
 * NULL, ndev entries): each device's HIP-event time. */
XSKNF_GPU_API int xsknf_gpu_multi_process(struct xsknf_gpu_multi *m, uint32_t ingress_ifindex,
		const struct xsknf_csum_opts *opts, uint32_t frame_len_max, uint32_t frame_len_mean, float *ms);
/* The XSKNF_GPU_MULTI_COUNTERS counters of every shard, summed over the devices
 * by ncclAllReduce (the root's copy, to host memory).  -EOPNOTSUPP after a
 * packed scatter (a packed shard no longer holds its frames' UMEM offsets,
 * which the weighted sum needs; its results come back by _return). */
XSKNF_GPU_API int xsknf_gpu_multi_counters(struct xsknf_gpu_multi *m, uint64_t *out);
/* As xsknf_gpu_multi_scatter, moving only the frames' bytes: on the root a
 * kernel copies each shard's frames into 16-byte aligned slots of a packed
 * buffer (a frame keeps its address mod 16; the bytes that share its first and
 * last 16-byte chunk travel with it), and each shard receives its packed bytes
 * plus descriptors that address them (aligned-mode addresses; descriptors
 * outside the UMEM keep their length and get an address past any span).  The
 * root's own shard is packed straight into its shard buffer (its descriptors
 * still go as a send to itself).  A UMEM of 2 KiB chunks holding IMIX frames
 * moves ~1/5 of its span bytes.
 * seconds (may be NULL): the packing and the moves. */
XSKNF_GPU_API int xsknf_gpu_multi_scatter_packed(struct xsknf_gpu_multi *m, int root, const uint8_t *umem,
		uint64_t umem_size, const struct xsknf_gpu_desc *descs, uint64_t n, double *seconds);
/* The whole batch's results back to the root, after either scatter: every
 * device runs the summing pass over its shard in records-only mode (fused_stores
 * 3: the shard is only read), sends its 4-byte record / verdict per frame to
 * the root into verdicts[0..n) (device memory on the root, the scatter's frame
 * order), and a kernel on the root writes each record's check into `umem` (the
 * root UMEM the scatter read, at the frame the caller's descriptor names) and
 * turns it into the forward verdict.  `umem` and `verdicts` then hold what one
 * device's xsknf_gpu_checksum_batch over the whole batch leaves.  -EBUSY when
 * xsknf_gpu_multi_process has checksummed the shards in place since the
 * scatter (a second pass is not the first: a frame whose UDP header overlaps
 * its IP addresses sums the check the first wrote); scatter again.  ms (may be
 * NULL, ndev entries): each device's summing pass, HIP events; seconds (may be
 * NULL): the whole return. */
XSKNF_GPU_API int xsknf_gpu_multi_return(struct xsknf_gpu_multi *m, uint32_t ingress_ifindex,
		const struct xsknf_csum_opts *opts, uint32_t frame_len_max, uint32_t frame_len_mean, uint8_t *umem,
		int32_t *verdicts, float *ms, double *seconds);
XSKNF_GPU_API int xsknf_gpu_multi_shard_info(const struct xsknf_gpu_multi *m, int shard,
		struct xsknf_gpu_shard_info *info);
/* Copy shard `shard`'s UMEM span (span_hi - span_lo bytes), its rebased
 * descriptors and its verdicts to host memory (any of them may be NULL). */
XSKNF_GPU_API int xsknf_gpu_multi_fetch(const struct xsknf_gpu_multi *m, int shard, uint8_t *umem_out,
		struct xsknf_gpu_desc *descs_out, int32_t *verdicts_out);
XSKNF_GPU_API int xsknf_gpu_multi_destroy(struct xsknf_gpu_multi *m);

/* Text of the last HIP error seen by this library, on any thread (a copy
 * private to the calling thread). */
XSKNF_GPU_API const char *xsknf_gpu_last_error(void);

/* Pool guard of the current device (synchronizes it first): how many waves of
 * the pooled split kernel found a unit of their block that no wave claimed
 * (its frames left unsummed).  The launch's grid bound makes this unreachable;
 * a nonzero count is a library bug.  reset != 0 zeroes the count after reading.
 * No reference counterpart (a device-side invariant check for tests and
 * monitoring). */
XSKNF_GPU_API int xsknf_gpu_pool_guard_trips(uint32_t *trips, int reset);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* XSKNF_GPU_H */

// xsknf_rt.c -- the AF_XDP worker runtime around the checksummer hot path.
//
// Mirrors the reference library (src/xsknf.c): per-worker UMEM with 4096
// frames per socket, one AF_XDP socket per (worker, interface), a worker
// thread pinned per CPU that loops over rx batches, recycles dropped frames to
// the fill ring and redirected ones through tx / completion.  The per-frame
// callback loop at src/xsknf.c:654-672 (and :500-522) is where the GPU batch
// hook (xsknf_set_batch_processor) takes over: one call per rx batch.
//
// Written on raw linux/if_xdp.h: XDP_UMEM_REG / ring setsockopts / mmaps /
// bind, a built-in XSKMAP-redirect XDP program (the role libxdp's default
// program plays for the reference, :137-141) and rtnetlink attach.  See
// include/xsknf.h for the deliberate differences from the reference.
#define _GNU_SOURCE

#include "../../include/xsknf.h"

#include <errno.h>
#include <getopt.h>
#include <linux/bpf.h>
#include <linux/if_link.h>
#include <net/if.h>
#include <poll.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "rt_netlink.h"
#include "xsk_ring.h"

#pragma weak xsknf_packet_processor

#ifndef SOL_XDP
#define SOL_XDP 283
#endif
#ifndef AF_XDP
#define AF_XDP 44
#endif
#ifndef SO_BUSY_POLL
#define SO_BUSY_POLL 46
#endif
#ifndef SO_PREFER_BUSY_POLL
#define SO_PREFER_BUSY_POLL 69
#endif
#ifndef SO_BUSY_POLL_BUDGET
#define SO_BUSY_POLL_BUDGET 70
#endif

// UMEM geometry of the reference (src/xsknf.c:29-37): frame addresses are
// | owner socket | frame id | in-frame offset |.
#define FRAMES_PER_SOCKET_SHIFT 12
#define FRAMES_PER_SOCKET (1u << FRAMES_PER_SOCKET_SHIFT)
#define DEFAULT_FRAME_SIZE 4096          // XSK_UMEM__DEFAULT_FRAME_SIZE
#define RING_DESCS 2048                  // XSK_RING_{CONS,PROD}__DEFAULT_NUM_DESCS
#define FILL_DESCS (2 * RING_DESCS)      // umem fill_size, src/xsknf.c:929
#define DEFAULT_BIND_FLAGS XDP_USE_NEED_WAKEUP
#define POLL_TIMEOUT_MS 1000
#define XDP_HEADROOM 256                 // XDP_PACKET_HEADROOM
#define UNALIGNED_SHIFT 48
#define UNALIGNED_MASK ((1ull << UNALIGNED_SHIFT) - 1)

struct pkt_info {
	uint64_t addr;
	uint32_t len;
};

struct emu_ring_mem {                    // shared indices on separate lines
	uint32_t producer __attribute__((aligned(64)));
	uint32_t consumer __attribute__((aligned(64)));
	uint32_t flags __attribute__((aligned(64)));
	uint8_t entries[] __attribute__((aligned(64)));
};

struct worker;

struct xsk_sock {
	struct worker *worker;
	unsigned if_idx;
	int fd;                              // -1 on an emulated queue
	uint32_t bind_flags;
	uint8_t *buffer;                     // UMEM this socket's frames live in
	struct xsk_ring rx, tx, fq, cq;      // the application's views
	void *map[4];
	size_t map_len[4];
	struct xsknf_socket_stats stats;
	uint32_t outstanding_tx;
	// emulated queues: ring storage and the kernel-side views
	struct emu_ring_mem *emu[4];
	struct xsk_ring k_rx, k_tx, k_fq, k_cq;
	unsigned long emu_rx_full, emu_fill_empty;
};

#define PEND_RING (XSKNF_MAX_HOOK_DEPTH + 1)

struct worker {
	unsigned id;
	pthread_t thread;
	int started;
	int err;
	struct xsk_sock *xsks;
	uint8_t *buffer;                     // zero-copy UMEM
	uint8_t *copy_buffer;                // copy-mode UMEM
	int umem_fd, copy_umem_fd;           // socket that registered each UMEM
	// per-batch scratch, sized by batch_size at init
	struct xdp_desc *descs;
	int32_t *verdicts;
	// two-phase hook: the batches in flight, oldest first, a ring of PEND_RING
	// (up to depth + 1 between a submit and the completion it triggers; each
	// with its own descriptor / verdict arrays, which swap with descs /
	// verdicts above when a batch is submitted)
	struct pending {
		struct xdp_desc *descs;
		int32_t *verdicts;
		uint32_t n;
		unsigned ifindex;            // the rx interface it came from
		uint64_t ticket;
	} pend[PEND_RING];
	unsigned pend_head, pend_count;
	struct pkt_info *to_drop;
	struct pkt_info *to_tx;              // [num_interfaces][batch_size]
	uint32_t *ntx;
	uint64_t *to_fill;                   // [num_interfaces][batch_size]
	uint32_t *nfill;
} __attribute__((aligned(64)));

struct iface {
	int ifindex;
	int emulated;
	int map_fd;
	int prog_fd;
	int attached;
};

static struct xsknf_config conf;
static const struct xsknf_config default_conf = {
	.working_mode = MODE_AF_XDP,
	.xsk_frame_size = DEFAULT_FRAME_SIZE,
	.batch_size = 64,
	.workers = 1,
	.xdp_flags = XDP_FLAGS_UPDATE_IF_NOEXIST,
};
static int initialised;
static int stop_flag;
static size_t umem_bufsize;
static uint64_t socket_span;             // bytes of UMEM owned by one socket
static struct worker *workers;
static struct iface *ifaces;
static xsknf_packet_processor_fn packet_fn;
static xsknf_batch_processor_fn batch_fn;
static void *batch_user;
static xsknf_batch_submit_fn submit_fn;
static xsknf_batch_complete_fn complete_fn;
static unsigned hook_depth = 1;          // batches a worker keeps in flight (two-phase hook)

static inline uint64_t addr_offset(uint64_t addr)
{
	// xsk_umem__add_offset_to_addr (src/xsknf.c:659); identity in aligned mode
	return (addr & UNALIGNED_MASK) + (addr >> UNALIGNED_SHIFT);
}

static int is_emulated(const char *name)
{
	return strncmp(name, "emu", 3) == 0;
}

/* ---- the XDP side: XSKMAP + redirect program, attached over rtnetlink ---- */

static long sys_bpf(int cmd, union bpf_attr *attr)
{
	return syscall(__NR_bpf, cmd, attr, sizeof(*attr));
}

// xdp: return bpf_redirect_map(&xsks, ctx->rx_queue_index, XDP_PASS);
static int load_redirect_prog(int map_fd)
{
	struct bpf_insn prog[] = {
		// r2 = *(u32 *)(r1 + offsetof(struct xdp_md, rx_queue_index))
		{.code = BPF_LDX | BPF_MEM | BPF_W, .dst_reg = BPF_REG_2, .src_reg = BPF_REG_1,
		 .off = 16},
		// r1 = map (ld_imm64, two slots)
		{.code = BPF_LD | BPF_DW | BPF_IMM, .dst_reg = BPF_REG_1,
		 .src_reg = BPF_PSEUDO_MAP_FD, .imm = map_fd},
		{0},
		// r3 = XDP_PASS: the action when the queue has no socket
		{.code = BPF_ALU64 | BPF_MOV | BPF_K, .dst_reg = BPF_REG_3, .imm = XDP_PASS},
		{.code = BPF_JMP | BPF_CALL, .imm = BPF_FUNC_redirect_map},
		{.code = BPF_JMP | BPF_EXIT},
	};
	static const char license[] = "GPL";
	union bpf_attr a;
	memset(&a, 0, sizeof(a));
	a.prog_type = BPF_PROG_TYPE_XDP;
	a.insns = (uintptr_t)prog;
	a.insn_cnt = sizeof(prog) / sizeof(prog[0]);
	a.license = (uintptr_t)license;
	const long fd = sys_bpf(BPF_PROG_LOAD, &a);
	return fd < 0 ? -errno : (int)fd;
}

static int setup_xdp(struct iface *f)
{
	union bpf_attr a;
	memset(&a, 0, sizeof(a));
	a.map_type = BPF_MAP_TYPE_XSKMAP;
	a.key_size = sizeof(int);
	a.value_size = sizeof(int);
	a.max_entries = XSKNF_MAX_WORKERS;
	long fd = sys_bpf(BPF_MAP_CREATE, &a);
	if (fd < 0)
		return -errno;
	f->map_fd = (int)fd;
	const int prog = load_redirect_prog(f->map_fd);
	if (prog < 0)
		return prog;
	f->prog_fd = prog;
	const int rc = xsknf_nl_set_xdp(f->ifindex, f->prog_fd, conf.xdp_flags);
	if (rc)
		return rc;
	f->attached = 1;
	return 0;
}

static int map_insert(int map_fd, int key, int sock_fd)
{
	union bpf_attr a;
	memset(&a, 0, sizeof(a));
	a.map_fd = map_fd;
	a.key = (uintptr_t)&key;
	a.value = (uintptr_t)&sock_fd;
	a.flags = BPF_ANY;
	return sys_bpf(BPF_MAP_UPDATE_ELEM, &a) ? -errno : 0;
}

/* ---- sockets ---- */

static void ring_view(struct xsk_ring *r, void *base, const struct xdp_ring_offset *o,
		uint32_t size)
{
	r->producer = (uint32_t *)((uint8_t *)base + o->producer);
	r->consumer = (uint32_t *)((uint8_t *)base + o->consumer);
	r->flags = (uint32_t *)((uint8_t *)base + o->flags);
	r->entries = (uint8_t *)base + o->desc;
	r->size = size;
	r->mask = size - 1;
}

static int open_kernel_socket(struct xsk_sock *s, int ifindex, unsigned queue, int *umem_fd)
{
	int fd = socket(AF_XDP, SOCK_RAW | SOCK_CLOEXEC, 0);
	if (fd < 0)
		return -errno;
	s->fd = fd;
	const int first = *umem_fd < 0;
	if (first) {
		struct xdp_umem_reg mr = {
			.addr = (uintptr_t)s->buffer,
			.len = umem_bufsize,
			.chunk_size = (uint32_t)conf.xsk_frame_size,
			.headroom = 0,
			.flags = conf.unaligned_chunks ? XDP_UMEM_UNALIGNED_CHUNK_FLAG : 0,
		};
		if (setsockopt(fd, SOL_XDP, XDP_UMEM_REG, &mr, sizeof(mr)))
			return -errno;
	}
	const int fill = FILL_DESCS, comp = RING_DESCS, rxn = RING_DESCS, txn = RING_DESCS;
	if (setsockopt(fd, SOL_XDP, XDP_UMEM_FILL_RING, &fill, sizeof(fill)) ||
	    setsockopt(fd, SOL_XDP, XDP_UMEM_COMPLETION_RING, &comp, sizeof(comp)) ||
	    setsockopt(fd, SOL_XDP, XDP_RX_RING, &rxn, sizeof(rxn)) ||
	    setsockopt(fd, SOL_XDP, XDP_TX_RING, &txn, sizeof(txn)))
		return -errno;
	struct xdp_mmap_offsets off;
	socklen_t optlen = sizeof(off);
	if (getsockopt(fd, SOL_XDP, XDP_MMAP_OFFSETS, &off, &optlen))
		return -errno;
	const struct {
		const struct xdp_ring_offset *o;
		uint32_t n;
		size_t esz;
		off_t pgoff;
		struct xsk_ring *r;
	} rings[4] = {
		{&off.rx, RING_DESCS, sizeof(struct xdp_desc), XDP_PGOFF_RX_RING, &s->rx},
		{&off.tx, RING_DESCS, sizeof(struct xdp_desc), XDP_PGOFF_TX_RING, &s->tx},
		{&off.fr, FILL_DESCS, sizeof(uint64_t), XDP_UMEM_PGOFF_FILL_RING, &s->fq},
		{&off.cr, RING_DESCS, sizeof(uint64_t), XDP_UMEM_PGOFF_COMPLETION_RING, &s->cq},
	};
	for (int i = 0; i < 4; ++i) {
		const size_t len = rings[i].o->desc + rings[i].n * rings[i].esz;
		void *m = mmap(NULL, len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd,
				rings[i].pgoff);
		if (m == MAP_FAILED)
			return -errno;
		s->map[i] = m;
		s->map_len[i] = len;
		ring_view(rings[i].r, m, rings[i].o, rings[i].n);
	}
	struct sockaddr_xdp sxdp = {
		.sxdp_family = AF_XDP,
		.sxdp_ifindex = (uint32_t)ifindex,
		.sxdp_queue_id = queue,
	};
	if (first) {
		sxdp.sxdp_flags = (uint16_t)s->bind_flags;
	} else {
		// sharers inherit copy / zero-copy / need-wakeup from the owner
		sxdp.sxdp_flags = XDP_SHARED_UMEM;
		sxdp.sxdp_shared_umem_fd = (uint32_t)*umem_fd;
	}
	if (bind(fd, (struct sockaddr *)&sxdp, sizeof(sxdp)))
		return -errno;
	if (first)
		*umem_fd = fd;

	if (conf.busy_poll && !(s->bind_flags & XDP_COPY)) {   // src/xsknf.c:145-161
		int v = 1;
		if (setsockopt(fd, SOL_SOCKET, SO_PREFER_BUSY_POLL, &v, sizeof(v)))
			return -errno;
		v = 20;
		if (setsockopt(fd, SOL_SOCKET, SO_BUSY_POLL, &v, sizeof(v)))
			return -errno;
		v = (int)conf.batch_size;
		if (setsockopt(fd, SOL_SOCKET, SO_BUSY_POLL_BUDGET, &v, sizeof(v)))
			return -errno;
	}
	return 0;
}

static int open_emulated_socket(struct xsk_sock *s)
{
	const struct {
		uint32_t n;
		size_t esz;
		struct xsk_ring *app, *kern;
	} rings[4] = {
		{RING_DESCS, sizeof(struct xdp_desc), &s->rx, &s->k_rx},
		{RING_DESCS, sizeof(struct xdp_desc), &s->tx, &s->k_tx},
		{FILL_DESCS, sizeof(uint64_t), &s->fq, &s->k_fq},
		{RING_DESCS, sizeof(uint64_t), &s->cq, &s->k_cq},
	};
	s->fd = -1;
	for (int i = 0; i < 4; ++i) {
		struct emu_ring_mem *m = aligned_alloc(64, sizeof(*m) + rings[i].n * rings[i].esz);
		if (!m)
			return -ENOMEM;
		memset(m, 0, sizeof(*m));
		s->emu[i] = m;
		for (int side = 0; side < 2; ++side) {
			struct xsk_ring *r = side ? rings[i].kern : rings[i].app;
			r->producer = &m->producer;
			r->consumer = &m->consumer;
			r->flags = &m->flags;
			r->entries = m->entries;
			r->size = rings[i].n;
			r->mask = rings[i].n - 1;
		}
	}
	return 0;
}

// the application-side index caches, once the rings exist
static void init_views(struct xsk_sock *s)
{
	ring_cons_init(&s->rx);
	ring_prod_init(&s->tx);
	ring_prod_init(&s->fq);
	ring_cons_init(&s->cq);
	if (s->fd < 0) {
		ring_prod_init(&s->k_rx);
		ring_cons_init(&s->k_tx);
		ring_cons_init(&s->k_fq);
		ring_prod_init(&s->k_cq);
	}
}

// populate the fill ring with the socket's own 4096 frames (src/xsknf.c:163-171)
static int populate_fill(struct xsk_sock *s)
{
	uint32_t idx;
	if (ring_reserve(&s->fq, FRAMES_PER_SOCKET, &idx) != FRAMES_PER_SOCKET)
		return -ENOSPC;
	const uint64_t first = (uint64_t)s->if_idx * FRAMES_PER_SOCKET;
	for (uint32_t i = 0; i < FRAMES_PER_SOCKET; i++)
		*ring_addr(&s->fq, idx + i) = (first + i) * (uint64_t)conf.xsk_frame_size;
	ring_submit(&s->fq, FRAMES_PER_SOCKET);
	return 0;
}

/* ---- the datapath (src/xsknf.c:397-742) ---- */

static void kick_tx(struct xsk_sock *s)
{
	if (s->fd < 0)
		return;
	if (sendto(s->fd, NULL, 0, MSG_DONTWAIT, NULL, 0) >= 0)
		return;
	if (errno == ENOBUFS || errno == EAGAIN || errno == EBUSY || errno == ENETDOWN)
		return;
	s->worker->err = -errno;
}

static inline int needs_tx_trigger(const struct xsk_sock *s)
{
	return (s->bind_flags & XDP_COPY) ||
	       (!conf.poll && !conf.busy_poll && ring_needs_wakeup(&s->tx));
}

// Reserve on the fill ring for frames we hold, which must fit: the ring has a
// slot for every frame of the socket.  The kernel publishes its fill consumer
// index after the rx producer (xsk_flush), so a frame can be seen on rx while
// its fill slot still counts as used: wait for the index instead of failing
// (the reference exits there, src/xsknf.c:690-693).
static int reserve_exact(struct xsk_ring *r, uint32_t n, uint32_t *idx)
{
	for (long spin = 0; spin < (1L << 24); spin++) {
		if (ring_reserve(r, n, idx) == n)
			return 0;
		__builtin_ia32_pause();
	}
	return -ENOSPC;
}

// complete_tx_1if (src/xsknf.c:587-628): completions go back to the fill ring
static int complete_tx_1if(struct xsk_sock *s)
{
	if (!s->outstanding_tx)
		return 0;
	if (needs_tx_trigger(s)) {
		s->stats.tx_trigger_sendtos++;
		kick_tx(s);
	}
	const uint32_t want = s->outstanding_tx > conf.batch_size ? conf.batch_size : s->outstanding_tx;
	uint32_t idx_cq, idx_fq;
	const uint32_t sent = ring_peek(&s->cq, want, &idx_cq);
	if (!sent)
		return 0;
	s->stats.tx_npkts += sent;
	if (reserve_exact(&s->fq, sent, &idx_fq))
		return -ENOSPC;
	for (uint32_t i = 0; i < sent; i++)
		*ring_addr(&s->fq, idx_fq + i) = *ring_addr(&s->cq, idx_cq + i);
	ring_submit(&s->fq, sent);
	ring_release(&s->cq, sent);
	s->outstanding_tx -= sent;
	return 0;
}

// complete_tx (src/xsknf.c:413-474): completions go to the owner socket's fill ring
static int complete_tx(struct xsk_sock *xsks, unsigned ifindex)
{
	struct xsk_sock *tx = &xsks[ifindex];
	struct worker *w = tx->worker;
	if (!tx->outstanding_tx)
		return 0;
	if (needs_tx_trigger(tx)) {
		tx->stats.tx_trigger_sendtos++;
		kick_tx(tx);
	}
	const uint32_t want = tx->outstanding_tx > conf.batch_size ? conf.batch_size : tx->outstanding_tx;
	uint32_t idx;
	const uint32_t sent = ring_peek(&tx->cq, want, &idx);
	if (!sent)
		return 0;
	memset(w->nfill, 0, sizeof(uint32_t) * conf.num_interfaces);
	for (uint32_t i = 0; i < sent; i++) {
		const uint64_t addr = *ring_addr(&tx->cq, idx + i);
		uint64_t owner = addr_offset(addr) / socket_span;
		if (owner >= conf.num_interfaces)
			owner = ifindex;
		w->to_fill[owner * conf.batch_size + w->nfill[owner]++] = addr;
	}
	ring_release(&tx->cq, sent);
	tx->stats.tx_npkts += sent;
	for (unsigned i = 0; i < conf.num_interfaces; i++) {
		if (!w->nfill[i])
			continue;
		if (reserve_exact(&xsks[i].fq, w->nfill[i], &idx))
			return -ENOSPC;
		for (uint32_t j = 0; j < w->nfill[i]; j++)
			*ring_addr(&xsks[i].fq, idx + j) = w->to_fill[i * conf.batch_size + j];
		ring_submit(&xsks[i].fq, w->nfill[i]);
	}
	tx->outstanding_tx -= sent;
	return 0;
}

// Take the rcvd descriptors at ring index idx out of the rx ring into
// w->descs (the frames stay the worker's until they go to a tx or fill ring).
static void take_rx(struct xsk_sock *rx, uint32_t idx, uint32_t rcvd)
{
	struct worker *w = rx->worker;
	for (uint32_t i = 0; i < rcvd; i++)
		w->descs[i] = *ring_desc(&rx->rx, idx + i);
	ring_release(&rx->rx, rcvd);
	rx->stats.rx_npkts += rcvd;
}

// run the NF over w->descs[0, rcvd): verdicts[] out
static int run_nf(struct xsk_sock *rx, uint32_t rcvd, unsigned ingress)
{
	struct worker *w = rx->worker;
	if (batch_fn)
		return batch_fn(batch_user, w->id, rx->buffer, umem_bufsize, w->descs, rcvd, ingress,
				w->verdicts);
	xsknf_packet_processor_fn fn = packet_fn ? packet_fn : xsknf_packet_processor;
	for (uint32_t i = 0; i < rcvd; i++) {
		const struct xdp_desc *d = &w->descs[i];
		w->verdicts[i] = fn(rx->buffer + addr_offset(d->addr), d->len, ingress);
	}
	return 0;
}

static void rx_empty(struct xsk_sock *s)
{
	if (s->fd >= 0 && !(s->bind_flags & XDP_COPY) &&
	    (conf.busy_poll || ring_needs_wakeup(&s->fq))) {
		s->stats.rx_empty_polls++;
		recvfrom(s->fd, NULL, 0, MSG_DONTWAIT, NULL, NULL);
	}
}

static int recycle_pkts(struct xsk_sock *s, const struct pkt_info *p, uint32_t n)
{
	uint32_t idx;
	if (!n)
		return 0;
	if (reserve_exact(&s->fq, n, &idx))
		return -ENOSPC;
	for (uint32_t i = 0; i < n; i++)
		*ring_addr(&s->fq, idx + i) = p[i].addr;
	ring_submit(&s->fq, n);
	return 0;
}

static int recycle_drops(struct xsk_sock *s, uint32_t ndrop)
{
	return recycle_pkts(s, s->worker->to_drop, ndrop);
}

// A stop (or a worker error) while the tx ring is full: the frames that were to
// be sent go back to the rx socket's fill ring, so no frame leaks from the
// socket's budget and the sockets can run again after xsknf_start_workers().
static int abandon_tx(struct xsk_sock *rx, const struct pkt_info *p, uint32_t n)
{
	const int rc = recycle_pkts(rx, p, n);
	return rx->worker->err ? rx->worker->err : rc;
}

// The tx / fill half of process_batch_1if (src/xsknf.c:674-714) for a batch
// whose verdicts are known.
static int dispose_1if(struct xsk_sock *s, const struct xdp_desc *descs, const int32_t *verdicts,
		       uint32_t rcvd)
{
	struct worker *w = s->worker;
	uint32_t ndrop = 0, ntx = 0, idx;
	int rc;
	for (uint32_t i = 0; i < rcvd; i++) {
		struct pkt_info p = {descs[i].addr, descs[i].len};
		if (verdicts[i] == -1)
			w->to_drop[ndrop++] = p;
		else
			w->to_tx[ntx++] = p;    // any other verdict: the one tx queue
	}
	if ((rc = recycle_drops(s, ndrop)))
		return rc;
	if (ntx) {
		while (ring_reserve(&s->tx, ntx, &idx) != ntx) {
			if ((rc = complete_tx_1if(s)))
				return rc;
			if (conf.busy_poll || ring_needs_wakeup(&s->tx)) {
				s->stats.tx_wakeup_sendtos++;
				kick_tx(s);
			}
			if (w->err || __atomic_load_n(&stop_flag, __ATOMIC_RELAXED))
				return abandon_tx(s, w->to_tx, ntx);
		}
		for (uint32_t i = 0; i < ntx; i++) {
			struct xdp_desc *d = ring_desc(&s->tx, idx + i);
			d->addr = w->to_tx[i].addr;
			d->len = w->to_tx[i].len;
			d->options = 0;
		}
		ring_submit(&s->tx, ntx);
		s->outstanding_tx += ntx;
	}
	return 0;
}

// The tx / fill half of process_batch (src/xsknf.c:500-585): per-destination
// tx, cross-UMEM copies.
static int dispose_multi(struct xsk_sock *xsks, unsigned ifindex, const struct xdp_desc *descs,
			 const int32_t *verdicts, uint32_t rcvd)
{
	struct xsk_sock *rx = &xsks[ifindex];
	struct worker *w = rx->worker;
	const unsigned nif = conf.num_interfaces;
	uint32_t ndrop = 0, idx;
	int rc;
	memset(w->ntx, 0, sizeof(uint32_t) * nif);
	for (uint32_t i = 0; i < rcvd; i++) {
		struct pkt_info p = {descs[i].addr, descs[i].len};
		const int32_t v = verdicts[i];
		if (v < 0 || (unsigned)v >= nif)
			w->to_drop[ndrop++] = p;
		else
			w->to_tx[(unsigned)v * conf.batch_size + w->ntx[v]++] = p;
	}
	if ((rc = recycle_drops(rx, ndrop)))
		return rc;
	for (unsigned i = 0; i < nif; i++) {
		const uint32_t n = w->ntx[i];
		if (!n)
			continue;
		struct xsk_sock *tx = &xsks[i];
		while (ring_reserve(&tx->tx, n, &idx) != n) {
			// reap the rx interface's completions (as src/xsknf.c:554 does) and
			// the destination's own: with its completion ring full the kernel
			// cannot consume its tx ring, and the wait would never end
			if ((rc = complete_tx(xsks, ifindex)))
				return rc;
			if (i != ifindex && (rc = complete_tx(xsks, i)))
				return rc;
			if (conf.busy_poll || ring_needs_wakeup(&tx->tx)) {
				tx->stats.tx_wakeup_sendtos++;
				kick_tx(tx);
			}
			if (w->err || __atomic_load_n(&stop_flag, __ATOMIC_RELAXED)) {
				// this destination's frames and every later one's, each to
				// its owner's fill ring (as complete_tx recycles them)
				for (unsigned k = i; k < nif; k++) {
					const struct pkt_info *p = &w->to_tx[k * conf.batch_size];
					for (uint32_t j = 0; j < w->ntx[k]; j++) {
						uint64_t owner = addr_offset(p[j].addr) / socket_span;
						if (owner >= nif)
							owner = ifindex;
						const int r2 = recycle_pkts(&xsks[owner], &p[j], 1);
						if (r2 && !rc)
							rc = r2;
					}
				}
				return w->err ? w->err : rc;
			}
		}
		const struct pkt_info *p = &w->to_tx[i * conf.batch_size];
		for (uint32_t j = 0; j < n; j++) {
			if (rx->buffer != tx->buffer) {
				const uint64_t off = addr_offset(p[j].addr);
				memcpy(tx->buffer + off, rx->buffer + off, p[j].len);
			}
			struct xdp_desc *d = ring_desc(&tx->tx, idx + j);
			d->addr = p[j].addr;
			d->len = p[j].len;
			d->options = 0;
		}
		ring_submit(&tx->tx, n);
		tx->outstanding_tx += n;
	}
	return 0;
}

static int dispose(struct xsk_sock *xsks, unsigned ifindex, const struct xdp_desc *descs,
		   const int32_t *verdicts, uint32_t n)
{
	return conf.num_interfaces > 1 ? dispose_multi(xsks, ifindex, descs, verdicts, n)
				       : dispose_1if(&xsks[ifindex], descs, verdicts, n);
}

// The oldest batch in flight (two-phase hook): wait for its verdicts, then route it.
static int finish_oldest(struct worker *w)
{
	if (!w->pend_count)
		return 0;
	struct pending *b = &w->pend[w->pend_head];
	w->pend_head = (w->pend_head + 1) % PEND_RING;
	w->pend_count--;
	struct xsk_sock *rx = &w->xsks[b->ifindex];
	int rc = complete_fn(batch_user, w->id, rx->buffer, b->ticket);
	if (rc) {
		// verdicts unknown: the frames go back to the rx socket's fill ring
		struct pkt_info *p = w->to_drop;
		for (uint32_t i = 0; i < b->n; i++)
			p[i] = (struct pkt_info){b->descs[i].addr, b->descs[i].len};
		recycle_pkts(rx, p, b->n);
		return rc;
	}
	return dispose(w->xsks, b->ifindex, b->descs, b->verdicts, b->n);
}

static int finish_all(struct worker *w)
{
	int rc = 0;
	while (w->pend_count) {
		const int r = finish_oldest(w);
		if (r && !rc)
			rc = r;
	}
	return rc;
}

// One rx batch of interface ifindex (process_batch_1if / process_batch,
// src/xsknf.c:630-714, :478-585).  With the two-phase hook the batch is
// submitted, and the oldest in flight is completed and routed once more than
// hook_depth are out.  *rcvd_any is set when a batch came in.
static int process_rx(struct xsk_sock *xsks, unsigned ifindex, int *rcvd_any)
{
	struct xsk_sock *rx = &xsks[ifindex];
	struct worker *w = rx->worker;
	int rc = conf.num_interfaces > 1 ? complete_tx(xsks, ifindex) : complete_tx_1if(rx);
	if (rc)
		return rc;
	uint32_t idx;
	const uint32_t rcvd = ring_peek(&rx->rx, conf.batch_size, &idx);
	if (!rcvd) {
		rx_empty(rx);
		return 0;
	}
	*rcvd_any = 1;
	take_rx(rx, idx, rcvd);
	if (!submit_fn) {
		if ((rc = run_nf(rx, rcvd, ifindex)))
			return rc;
		return dispose(xsks, ifindex, w->descs, w->verdicts, rcvd);
	}
	uint64_t ticket = 0;
	rc = submit_fn(batch_user, w->id, rx->buffer, umem_bufsize, w->descs, rcvd, ifindex, w->verdicts,
		       &ticket);
	if (rc) {
		struct pkt_info *p = w->to_drop;
		for (uint32_t i = 0; i < rcvd; i++)
			p[i] = (struct pkt_info){w->descs[i].addr, w->descs[i].len};
		recycle_pkts(rx, p, rcvd);
		return rc;
	}
	// the new batch joins the ones in flight; its arrays swap with a free slot's
	struct pending *b = &w->pend[(w->pend_head + w->pend_count) % PEND_RING];
	struct xdp_desc *d = b->descs;
	int32_t *v = b->verdicts;
	*b = (struct pending){w->descs, w->verdicts, rcvd, ifindex, ticket};
	w->descs = d;
	w->verdicts = v;
	w->pend_count++;
	// then the oldest is completed and routed once more than hook_depth are out
	return w->pend_count > hook_depth ? finish_oldest(w) : 0;
}

// worker_loop (src/xsknf.c:716-742)
static void *worker_loop(void *arg)
{
	struct worker *w = arg;
	struct pollfd fds[XSKNF_MAX_INTERFACES];
	while (!__atomic_load_n(&stop_flag, __ATOMIC_RELAXED) && !w->err) {
		if (conf.poll) {
			nfds_t nfds = 0;
			for (unsigned i = 0; i < conf.num_interfaces; i++) {
				w->xsks[i].stats.opt_polls++;
				if (w->xsks[i].fd < 0)
					continue;
				fds[nfds].fd = w->xsks[i].fd;
				fds[nfds].events = POLLIN;
				fds[nfds].revents = 0;
				nfds++;
			}
			// (batches in flight: no blocking poll, they are flushed below)
			if (nfds && poll(fds, nfds, w->pend_count ? 0 : POLL_TIMEOUT_MS) <= 0 && !w->pend_count)
				continue;
		}
		int rc = 0, rcvd_any = 0;
		for (unsigned i = 0; i < conf.num_interfaces && !rc; i++)
			rc = process_rx(w->xsks, i, &rcvd_any);
		// a pass with no traffic on any interface: the batches in flight are
		// completed and routed, not held back waiting for more
		if (!rc && !rcvd_any)
			rc = finish_all(w);
		if (rc && !w->err)
			w->err = rc;
	}
	// a batch still in flight is completed and routed (on a stop its tx frames
	// go back to the fill rings: dispose sees the stop)
	const int rc = finish_all(w);
	if (rc && !w->err)
		w->err = rc;
	return NULL;
}

/* ---- argument parsing ----
 * The library's command line is the reference's contract (src/xsknf.c:744-874):
 * the same short options ("i:pSf:ub:BM:w:"), long names and meanings, parsed up
 * to the `--` that starts the application's own options, and a process that
 * gets a bad option ends with status 1 after printing what was wrong and the
 * option summary.  The wording of the messages is this runtime's own. */

static const struct option long_options[] = {
	{"iface", required_argument, 0, 'i'},
	{"poll", no_argument, 0, 'p'},
	{"xdp-skb", no_argument, 0, 'S'},
	{"frame-size", required_argument, 0, 'f'},
	{"unaligned", no_argument, 0, 'u'},
	{"batch-size", required_argument, 0, 'b'},
	{"busy-poll", no_argument, 0, 'B'},
	{"mode", required_argument, 0, 'M'},
	{"workers", required_argument, 0, 'w'},
	{0, 0, 0, 0},
};

static const struct {
	const char *flags, *text;
} option_help[] = {
	{"-i, --iface=IF[:c|z]", "receive on interface IF (repeatable); :c forces copy mode, :z zero-copy"},
	{"-p, --poll", "wait for traffic with poll() instead of spinning"},
	{"-S, --xdp-skb", "attach the redirect program in generic (skb) mode"},
	{"-f, --frame-size=N", "UMEM chunk size in bytes (a power of two unless -u)"},
	{"-u, --unaligned", "unaligned chunk mode: frames at any UMEM offset"},
	{"-b, --batch-size=N", "rx/tx descriptors handled per ring pass"},
	{"-B, --busy-poll", "request busy polling on the sockets"},
	{"-M, --mode=MODE", "AF_XDP (the only mode this runtime runs), XDP or COMBINED"},
	{"-w, --workers=N", "worker threads, one rx queue each"},
};

static void __attribute__((noreturn)) bad_args(const char *fmt, const char *arg)
{
	if (fmt)
		fprintf(stderr, fmt, arg);
	fprintf(stderr, "xsknf library options (before `--`; frame size default %d, batch size default %u):\n",
		DEFAULT_FRAME_SIZE, default_conf.batch_size);
	for (size_t k = 0; k < sizeof(option_help) / sizeof(option_help[0]); k++)
		fprintf(stderr, "  %-24s %s\n", option_help[k].flags, option_help[k].text);
	exit(EXIT_FAILURE);
}

// "IF" or "IF:c" / "IF:z": the interface name (the suffix cut off in place) and its bind flags
static void add_interface(struct xsknf_config *config, char *spec)
{
	if (config->num_interfaces >= XSKNF_MAX_INTERFACES)
		bad_args("xsknf: more interfaces than XSKNF_MAX_INTERFACES (at '%s')\n", spec);
	uint32_t flags = DEFAULT_BIND_FLAGS;
	char *mode = strchr(spec, ':');
	if (mode) {
		if (!strcmp(mode + 1, "c"))
			flags |= XDP_COPY;
		else if (!strcmp(mode + 1, "z"))
			flags |= XDP_ZEROCOPY;
		else
			bad_args("xsknf: copy mode '%s' is neither c nor z\n", mode + 1);
		*mode = 0;
	}
	config->bind_flags[config->num_interfaces] = flags;
	config->interfaces[config->num_interfaces++] = spec;
}

static int working_mode_of(const char *name)
{
	static const struct {
		const char *name;
		int mode;
	} modes[] = {{"AF_XDP", MODE_AF_XDP}, {"XDP", MODE_XDP}, {"COMBINED", MODE_COMBINED}};
	for (size_t k = 0; k < sizeof(modes) / sizeof(modes[0]); k++)
		if (!strcmp(name, modes[k].name))
			return modes[k].mode;
	bad_args("xsknf: no working mode named '%s'\n", name);
}

int xsknf_parse_args(int argc, char **argv, struct xsknf_config *config)
{
	memcpy(config, &default_conf, sizeof(*config));
	snprintf(config->ebpf_filename, sizeof(config->ebpf_filename), "%s_kern.o", argv[0]);
	snprintf(config->xdp_progname, sizeof(config->xdp_progname), "handle_xdp");
	config->tc_progname[0] = 0;

	int c, option_index;
	while ((c = getopt_long(argc, argv, "i:pSf:ub:BM:w:", long_options, &option_index)) != -1) {
		switch (c) {
		case 'i': add_interface(config, optarg); break;
		case 'p': config->poll = 1; break;
		case 'S': config->xdp_flags |= XDP_FLAGS_SKB_MODE; break;
		case 'u': config->unaligned_chunks = 1; break;
		case 'f': config->xsk_frame_size = atoi(optarg); break;
		case 'b': config->batch_size = (uint32_t)atoi(optarg); break;
		case 'B': config->busy_poll = 1; break;
		case 'M': config->working_mode = working_mode_of(optarg); break;
		case 'w':
			config->workers = (unsigned)atoi(optarg);
			if (config->workers < 1)
				bad_args("xsknf: worker count '%s' is not a positive number\n", optarg);
			break;
		default:   // getopt has already said what it did not understand
			bad_args(NULL, NULL);
		}
	}
	if (config->num_interfaces == 0)
		bad_args("%sxsknf: no interface given (-i IF)\n", "");
	if (!(config->xdp_flags & XDP_FLAGS_SKB_MODE))
		config->xdp_flags |= XDP_FLAGS_DRV_MODE;
	const unsigned fs = (unsigned)config->xsk_frame_size;
	if (!config->unaligned_chunks && (fs & (fs - 1))) {
		char num[16];
		snprintf(num, sizeof(num), "%d", config->xsk_frame_size);
		bad_args("xsknf: frame size %s must be a power of two without -u\n", num);
	}
	return 0;
}

/* ---- lifecycle ---- */

static void release_socket(struct xsk_sock *s)
{
	for (int i = 0; i < 4; ++i) {
		if (s->map[i])
			munmap(s->map[i], s->map_len[i]);
		s->map[i] = NULL;
		free(s->emu[i]);
		s->emu[i] = NULL;
	}
	if (s->fd >= 0)
		close(s->fd);
	s->fd = -1;
}

static void release_all(void)
{
	if (workers) {
		for (unsigned w = 0; w < conf.workers; w++) {
			struct worker *wk = &workers[w];
			if (wk->xsks)
				for (unsigned i = 0; i < conf.num_interfaces; i++)
					release_socket(&wk->xsks[i]);
			if (wk->buffer)
				munmap(wk->buffer, umem_bufsize);
			if (wk->copy_buffer)
				munmap(wk->copy_buffer, umem_bufsize);
			free(wk->xsks);
			free(wk->descs);
			free(wk->verdicts);
			for (unsigned k = 0; k < PEND_RING; k++) {
				free(wk->pend[k].descs);
				free(wk->pend[k].verdicts);
			}
			free(wk->to_drop);
			free(wk->to_tx);
			free(wk->ntx);
			free(wk->to_fill);
			free(wk->nfill);
		}
		free(workers);
		workers = NULL;
	}
	if (ifaces) {
		for (unsigned i = 0; i < conf.num_interfaces; i++) {
			struct iface *f = &ifaces[i];
			if (f->attached)
				xsknf_nl_set_xdp(f->ifindex, -1, conf.xdp_flags);
			if (f->prog_fd >= 0)
				close(f->prog_fd);
			if (f->map_fd >= 0)
				close(f->map_fd);
		}
		free(ifaces);
		ifaces = NULL;
	}
	initialised = 0;
}

static uint8_t *map_umem(void)
{
	// hugepages for unaligned chunks, as the reference (src/xsknf.c:925-926); plain
	// pages if none are reserved (chunks then must not straddle a 4 KiB page)
	int flags = MAP_PRIVATE | MAP_ANONYMOUS;
	void *p = MAP_FAILED;
	if (conf.unaligned_chunks)
		p = mmap(NULL, umem_bufsize, PROT_READ | PROT_WRITE, flags | MAP_HUGETLB, -1, 0);
	if (p == MAP_FAILED)
		p = mmap(NULL, umem_bufsize, PROT_READ | PROT_WRITE, flags, -1, 0);
	return p == MAP_FAILED ? NULL : p;
}

static int init_worker(struct worker *w)
{
	const unsigned nif = conf.num_interfaces;
	const size_t b = conf.batch_size;
	w->umem_fd = w->copy_umem_fd = -1;
	w->xsks = calloc(nif, sizeof(*w->xsks));
	w->descs = calloc(b, sizeof(*w->descs));
	w->verdicts = calloc(b, sizeof(*w->verdicts));
	int pend_ok = 1;
	for (unsigned k = 0; k < PEND_RING; k++) {
		w->pend[k].descs = calloc(b, sizeof(*w->pend[k].descs));
		w->pend[k].verdicts = calloc(b, sizeof(*w->pend[k].verdicts));
		pend_ok &= w->pend[k].descs && w->pend[k].verdicts;
	}
	w->to_drop = calloc(b, sizeof(*w->to_drop));
	w->to_tx = calloc(b * nif, sizeof(*w->to_tx));
	w->ntx = calloc(nif, sizeof(*w->ntx));
	w->to_fill = calloc(b * nif, sizeof(*w->to_fill));
	w->nfill = calloc(nif, sizeof(*w->nfill));
	if (!w->xsks || !w->descs || !w->verdicts || !pend_ok || !w->to_drop || !w->to_tx || !w->ntx ||
	    !w->to_fill || !w->nfill)
		return -ENOMEM;
	for (unsigned i = 0; i < nif; i++)
		w->xsks[i].fd = -1;
	for (unsigned i = 0; i < nif; i++) {
		struct xsk_sock *s = &w->xsks[i];
		s->worker = w;
		s->if_idx = i;
		s->bind_flags = conf.bind_flags[i];
		const int copy = (s->bind_flags & XDP_COPY) != 0;
		uint8_t **buf = copy ? &w->copy_buffer : &w->buffer;
		if (!*buf && !(*buf = map_umem()))
			return -errno;
		s->buffer = *buf;
		int rc;
		if (ifaces[i].emulated) {
			rc = open_emulated_socket(s);
		} else {
			rc = open_kernel_socket(s, ifaces[i].ifindex, w->id,
					copy ? &w->copy_umem_fd : &w->umem_fd);
			if (!rc)
				rc = map_insert(ifaces[i].map_fd, (int)w->id, s->fd);
		}
		if (rc)
			return rc;
		init_views(s);
		if ((rc = populate_fill(s)))
			return rc;
	}
	return 0;
}

int xsknf_init(struct xsknf_config *config, struct bpf_object **bpf_obj)
{
	if (initialised || !config)
		return -EINVAL;
	if (bpf_obj)
		*bpf_obj = NULL;
	memcpy(&conf, config, sizeof(conf));
	if (conf.working_mode & MODE_XDP)
		return -EOPNOTSUPP;   // the NF's own eBPF object (src/xsknf.c:985-998)
	if (conf.num_interfaces < 1 || conf.num_interfaces > XSKNF_MAX_INTERFACES ||
	    conf.workers < 1 || conf.workers > XSKNF_MAX_WORKERS || conf.batch_size < 1 ||
	    conf.xsk_frame_size < 2 * XDP_HEADROOM)
		return -EINVAL;
	if (!(conf.working_mode & MODE_AF_XDP))
		return -EINVAL;
	if (!conf.unaligned_chunks && (conf.xsk_frame_size & (conf.xsk_frame_size - 1)))
		return -EINVAL;
	__atomic_store_n(&stop_flag, 0, __ATOMIC_RELAXED);
	initialised = 1;

	int rc = 0;
	ifaces = calloc(conf.num_interfaces, sizeof(*ifaces));
	if (!ifaces) {
		rc = -ENOMEM;
		goto fail;
	}
	for (unsigned i = 0; i < conf.num_interfaces; i++) {
		struct iface *f = &ifaces[i];
		f->map_fd = f->prog_fd = -1;
		if (!conf.interfaces[i]) {
			rc = -EINVAL;
			goto fail;
		}
		if (is_emulated(conf.interfaces[i])) {
			f->emulated = 1;
			continue;
		}
		f->ifindex = (int)if_nametoindex(conf.interfaces[i]);
		if (!f->ifindex) {
			fprintf(stderr, "ERROR: interface \"%s\" does not exist\n", conf.interfaces[i]);
			rc = -ENODEV;
			goto fail;
		}
	}
	// bind flags: skb mode forces copy; no explicit mode means zero-copy (src/xsknf.c:908-924)
	for (unsigned i = 0; i < conf.num_interfaces; i++) {
		if (conf.xdp_flags & XDP_FLAGS_SKB_MODE) {
			conf.bind_flags[i] &= ~XDP_ZEROCOPY;
			conf.bind_flags[i] |= XDP_COPY;
		}
		if (!(conf.bind_flags[i] & (XDP_COPY | XDP_ZEROCOPY)))
			conf.bind_flags[i] |= XDP_ZEROCOPY;
	}
	for (unsigned i = 0; i < conf.num_interfaces; i++)
		if (!ifaces[i].emulated && (rc = setup_xdp(&ifaces[i])))
			goto fail;

	socket_span = (uint64_t)FRAMES_PER_SOCKET * (uint64_t)conf.xsk_frame_size;
	umem_bufsize = socket_span * conf.num_interfaces;
	workers = calloc(conf.workers, sizeof(*workers));
	if (!workers) {
		rc = -ENOMEM;
		goto fail;
	}
	for (unsigned w = 0; w < conf.workers; w++)
		workers[w].id = w;
	for (unsigned w = 0; w < conf.workers; w++)
		if ((rc = init_worker(&workers[w])))
			goto fail;
	memcpy(config, &conf, sizeof(conf));
	return 0;
fail:
	release_all();
	return rc;
}

int xsknf_start_workers(void)
{
	if (!initialised)
		return -EINVAL;
	if (!submit_fn && !batch_fn && !packet_fn && !xsknf_packet_processor)
		return -ENOENT;   // no NF linked in and none registered
	__atomic_store_n(&stop_flag, 0, __ATOMIC_RELAXED);
	// worker i runs on the i-th CPU of the process's affinity set (src/xsknf.c:1049-1095)
	cpu_set_t set;
	int rc = pthread_getaffinity_np(pthread_self(), sizeof(set), &set);
	if (rc)
		return -rc;
	int cpus[CPU_SETSIZE], ncpu = 0;
	for (int i = 0; i < CPU_SETSIZE; i++)
		if (CPU_ISSET(i, &set))
			cpus[ncpu++] = i;
	if ((unsigned)ncpu < conf.workers) {
		fprintf(stderr, "ERROR: not enough CPUs to host all workers\n");
		return -EINVAL;
	}
	for (unsigned i = 0; i < conf.workers; i++) {
		struct worker *w = &workers[i];
		w->err = 0;
		rc = pthread_create(&w->thread, NULL, worker_loop, w);
		if (rc) {
			xsknf_stop_workers();
			return -rc;
		}
		w->started = 1;
		CPU_ZERO(&set);
		CPU_SET(cpus[i], &set);
		rc = pthread_setaffinity_np(w->thread, sizeof(set), &set);
		if (rc) {
			xsknf_stop_workers();
			return -rc;
		}
	}
	return 0;
}

int xsknf_stop_workers(void)
{
	if (!initialised)
		return 0;
	__atomic_store_n(&stop_flag, 1, __ATOMIC_RELAXED);
	int err = 0;
	for (unsigned i = 0; i < conf.workers; i++) {
		if (!workers[i].started)
			continue;
		pthread_join(workers[i].thread, NULL);
		workers[i].started = 0;
		if (!err)
			err = workers[i].err;
	}
	return err;
}

int xsknf_cleanup(void)
{
	if (!initialised)
		return 0;
	const int err = xsknf_stop_workers();
	release_all();
	return err;
}

static struct xsk_sock *sock_at(unsigned worker_idx, unsigned iface_idx)
{
	if (!initialised || worker_idx >= conf.workers || iface_idx >= conf.num_interfaces)
		return NULL;
	return &workers[worker_idx].xsks[iface_idx];
}

int xsknf_get_socket_stats(unsigned worker_idx, unsigned iface_idx, struct xsknf_socket_stats *stats)
{
	struct xsk_sock *s = sock_at(worker_idx, iface_idx);
	if (!s || !stats)
		return -EINVAL;
	if (s->fd >= 0) {
		// ring-level counters from the kernel (src/xsknf.c:83-106, optlen fixed)
		struct xdp_statistics x;
		memset(&x, 0, sizeof(x));
		socklen_t optlen = sizeof(x);
		if (getsockopt(s->fd, SOL_XDP, XDP_STATISTICS, &x, &optlen))
			return -errno;
		s->stats.rx_dropped_npkts = x.rx_dropped;
		s->stats.rx_invalid_npkts = x.rx_invalid_descs;
		s->stats.tx_invalid_npkts = x.tx_invalid_descs;
		if (optlen == sizeof(x)) {
			s->stats.rx_full_npkts = x.rx_ring_full;
			s->stats.rx_fill_empty_npkts = x.rx_fill_ring_empty_descs;
			s->stats.tx_empty_npkts = x.tx_ring_empty_descs;
		}
	} else {
		s->stats.rx_full_npkts = __atomic_load_n(&s->emu_rx_full, __ATOMIC_RELAXED);
		s->stats.rx_fill_empty_npkts = __atomic_load_n(&s->emu_fill_empty, __ATOMIC_RELAXED);
	}
	memcpy(stats, &s->stats, sizeof(*stats));
	return 0;
}

int xsknf_set_packet_processor(xsknf_packet_processor_fn fn)
{
	packet_fn = fn;
	return 0;
}

int xsknf_set_batch_processor(xsknf_batch_processor_fn fn, void *user)
{
	batch_fn = fn;
	batch_user = user;
	submit_fn = NULL;
	complete_fn = NULL;
	return 0;
}

int xsknf_set_batch_depth(unsigned depth)
{
	if (depth < 1 || depth > XSKNF_MAX_HOOK_DEPTH)
		return -EINVAL;
	hook_depth = depth;
	return 0;
}

int xsknf_set_batch_processor_async(xsknf_batch_submit_fn submit, xsknf_batch_complete_fn complete, void *user)
{
	if (!submit != !complete)
		return -EINVAL;
	submit_fn = submit;
	complete_fn = complete;
	batch_fn = NULL;
	batch_user = user;
	return 0;
}

int xsknf_get_umem(unsigned worker_idx, unsigned iface_idx, void **buffer, uint64_t *size)
{
	struct xsk_sock *s = sock_at(worker_idx, iface_idx);
	if (!s || !buffer || !size)
		return -EINVAL;
	*buffer = s->buffer;
	*size = umem_bufsize;
	return 0;
}

int xsknf_worker_error(unsigned worker_idx)
{
	if (!initialised || worker_idx >= conf.workers)
		return -EINVAL;
	return __atomic_load_n(&workers[worker_idx].err, __ATOMIC_RELAXED);
}

/* ---- emulated queues: the kernel's side ---- */

int xsknf_emu_deliver(unsigned worker_idx, unsigned iface_idx, const uint8_t *data,
		const uint32_t *lens, uint32_t n, uint32_t stride)
{
	struct xsk_sock *s = sock_at(worker_idx, iface_idx);
	if (!s || s->fd >= 0 || (n && (!data || !lens)))
		return -EINVAL;
	const uint64_t room = (uint64_t)conf.xsk_frame_size - XDP_HEADROOM;
	for (uint32_t i = 0; i < n; i++)
		if (lens[i] > room || lens[i] > stride)
			return -EINVAL;
	const uint32_t space = ring_prod_space(&s->k_rx, n);
	uint32_t fidx = 0, ridx = 0;
	const uint32_t m = ring_peek(&s->k_fq, n < space ? n : space, &fidx);
	if (m < n) {
		if (space < n)
			__atomic_fetch_add(&s->emu_rx_full, 1, __ATOMIC_RELAXED);
		else
			__atomic_fetch_add(&s->emu_fill_empty, 1, __ATOMIC_RELAXED);
	}
	if (!m)
		return 0;
	ring_reserve(&s->k_rx, m, &ridx);   // space >= m
	for (uint32_t i = 0; i < m; i++) {
		const uint64_t fa = *ring_addr(&s->k_fq, fidx + i);
		uint64_t base;
		struct xdp_desc *d = ring_desc(&s->k_rx, ridx + i);
		if (conf.unaligned_chunks) {
			base = addr_offset(fa);
			d->addr = base | ((uint64_t)XDP_HEADROOM << UNALIGNED_SHIFT);
		} else {
			base = fa & ~(uint64_t)(conf.xsk_frame_size - 1);
			d->addr = base + XDP_HEADROOM;
		}
		if (base + XDP_HEADROOM + lens[i] > umem_bufsize) {   // a bad fill address
			d->addr = 0;
			d->len = 0;
			d->options = 0;
			continue;
		}
		memcpy(s->buffer + base + XDP_HEADROOM, data + (size_t)i * stride, lens[i]);
		d->len = lens[i];
		d->options = 0;
	}
	ring_release(&s->k_fq, m);
	ring_submit(&s->k_rx, m);
	return (int)m;
}

int xsknf_emu_transmit(unsigned worker_idx, unsigned iface_idx, uint8_t *out, uint32_t *lens,
		uint32_t max, uint32_t stride)
{
	struct xsk_sock *s = sock_at(worker_idx, iface_idx);
	if (!s || s->fd >= 0 || (max && (!out || !lens)))
		return -EINVAL;
	const uint32_t space = ring_prod_space(&s->k_cq, max);
	uint32_t tidx = 0, cidx = 0;
	const uint32_t m = ring_peek(&s->k_tx, max < space ? max : space, &tidx);
	if (!m)
		return 0;
	ring_reserve(&s->k_cq, m, &cidx);
	for (uint32_t i = 0; i < m; i++) {
		const struct xdp_desc *d = ring_desc(&s->k_tx, tidx + i);
		const uint64_t off = addr_offset(d->addr);
		const uint32_t len = d->len < stride ? d->len : stride;
		lens[i] = d->len;
		if (off + len <= umem_bufsize)
			memcpy(out + (size_t)i * stride, s->buffer + off, len);
		*ring_addr(&s->k_cq, cidx + i) = d->addr;
	}
	ring_release(&s->k_tx, m);
	ring_submit(&s->k_cq, m);
	return (int)m;
}

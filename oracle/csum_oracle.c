/*
 * csum_oracle.c -- CPU restatement of the xsknf checksummer per-packet path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (xsknf_amd/, include/)
 * links, loads or calls this file.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it, and only as the checker / the
 * reported CPU baseline.
 *
 * What it restates (clean-room, from reading the reference):
 *   oracle_packet_processor()  <- examples/checksummer/checksummer_user.c:30-112
 *                                 (xsknf_packet_processor, "sane code" loop :92-103)
 *   oracle_process_batch()     <- src/xsknf.c:654-672 (per-frame loop of
 *                                 process_batch_1if), including the libxdp
 *                                 xsk_umem__add_offset_to_addr() translation
 *                                 (addr & (2^48-1)) + (addr >> 48) used at :659
 *
 * The per-word loop is kept literal (one wrapping u32 add per 16-bit word,
 * odd tail byte added as a low byte, ONE fold with the carry dropped) so that
 * it is an independent statement of the algorithm from the GPU kernel, which
 * uses the closed byte-parity form.
 *
 * Parity pin: the reference's own xsknf_packet_processor() is compiled here
 * from its verbatim text (oracle/ref_extract.sh + ref_harness.c ->
 * oracle/_ref/libcsum_ref.so, `make -C oracle ref`); tests/test_ref_pin.py
 * holds this restatement equal to it byte for byte on 20,000 randomized
 * frames and the known answers C1-C6, and tests/golden/ is its output.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

struct oracle_desc {            /* struct xdp_desc, linux/if_xdp.h */
	uint64_t addr;
	uint32_t len;
	uint32_t options;
};

struct oracle_opts {
	int32_t csum_iterations;    /* checksummer_user.c:25, default 1 */
	int32_t action;             /* checksummer_user.c:15-18,24: 0 REDIRECT, 1 DROP */
	uint32_t num_interfaces;    /* config.num_interfaces, checksummer_user.c:111 */
	uint32_t reserved;
};

static inline uint16_t ld16(const uint8_t *p)
{
	/* host (little-endian) load of two network-order bytes, as the
	 * reference's `*(uint16_t *)` dereferences do on x86 */
	uint16_t v;
	memcpy(&v, p, 2);
	return v;
}

int oracle_packet_processor(void *pkt, unsigned len, unsigned ingress_ifindex,
		const struct oracle_opts *o)
{
	uint8_t *f = (uint8_t *)pkt;
	uint8_t *end = f + len;

	/* :34-37 ethernet header must fit */
	if (f + 14 > end)
		return -1;
	/* :39-41 non-IPv4 frames go to iface 0, even in DROP mode */
	if (!(f[12] == 0x08 && f[13] == 0x00))
		return 0;
	/* :43-46 20-byte IPv4 header must fit (ihl not consulted here) */
	if (f + 34 > end)
		return -1;
	/* :48-50 non-UDP -> 0 */
	if (f[23] != 17)
		return 0;
	/* :52-55 udp header placed by the unvalidated ihl nibble */
	uint8_t *udp = f + 14 + ((f[14] & 0x0f) << 2);
	if (udp + 8 > end)
		return -1;

	/* :57-65 pseudo-header, read before the check field is cleared */
	uint32_t s = 0;
	s += ld16(f + 26);
	s += ld16(f + 28);
	s += ld16(f + 30);
	s += ld16(f + 32);
	s += (uint32_t)17 << 8;
	s += ld16(udp + 4);

	/* :68 */
	udp[6] = 0;
	udp[7] = 0;

	/* :92-103 */
	for (int it = 0; it < o->csum_iterations; it++) {
		uint8_t *p = udp;
		while (p + 2 <= end) {
			s += ld16(p);
			p += 2;
		}
		if (p + 1 <= end)
			s += *p;
	}

	/* :105-108 single fold, carry of the fold discarded */
	uint16_t c = (uint16_t)((uint16_t)s + (uint16_t)(s >> 16));
	c = (uint16_t)~c;
	memcpy(udp + 6, &c, 2);

	/* :110-111 */
	return o->action == 0 ?
		(int)((ingress_ifindex + 1) % o->num_interfaces) : -1;
}

static inline uint64_t umem_offset(uint64_t addr)
{
	return (addr & ((1ULL << 48) - 1)) + (addr >> 48);
}

/*
 * process_batch_1if()-shaped loop: frames are handed to the per-packet
 * function in rx batches of `batch` descriptors (src/xsknf.c:642,654-672).
 */
void oracle_process_batch(uint8_t *umem, const struct oracle_desc *descs,
		uint32_t n, uint32_t ingress, const struct oracle_opts *o,
		int32_t *verdicts, uint32_t batch)
{
	if (batch == 0)
		batch = 64;
	for (uint32_t b = 0; b < n; b += batch) {
		uint32_t rcvd = n - b < batch ? n - b : batch;
		for (uint32_t i = 0; i < rcvd; i++) {
			const struct oracle_desc *d = &descs[b + i];
			void *pkt = umem + umem_offset(d->addr);
			verdicts[b + i] = oracle_packet_processor(pkt, d->len,
					ingress, o);
		}
	}
}

/* ---- CPU baseline timing (bench.py cpu_baseline leg) ---------------- */

struct worker_arg {
	uint8_t *umem;
	const struct oracle_desc *descs;
	uint32_t lo, hi;
	const struct oracle_opts *o;
	int32_t *verdicts;
	int cpu;
	int reps;
};

static void *worker(void *p)
{
	struct worker_arg *a = p;
	if (a->cpu >= 0) {
		cpu_set_t set;
		CPU_ZERO(&set);
		CPU_SET(a->cpu, &set);
		pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
	}
	for (int r = 0; r < a->reps; r++)
		oracle_process_batch(a->umem, a->descs + a->lo, a->hi - a->lo, 0,
				a->o, a->verdicts + a->lo, 64);
	return NULL;
}

/*
 * Run `reps` passes of the batch loop over `n` frames, split contiguously
 * over `threads` pthreads (each pinned to the i-th CPU of the affinity mask
 * when pin == 1, the i-th from its end when pin == 2).  Returns wall seconds (CLOCK_MONOTONIC), or -1 on error.
 */
double oracle_time_batch(uint8_t *umem, const struct oracle_desc *descs,
		uint32_t n, const struct oracle_opts *o, int32_t *verdicts,
		int threads, int reps, int pin)
{
	if (threads < 1 || threads > 1024)
		return -1.0;
	pthread_t tid[threads];
	struct worker_arg args[threads];
	int cpus[threads];
	cpu_set_t mask;
	int ncpu = 0;
	if (pin && sched_getaffinity(0, sizeof(mask), &mask) == 0) {
		/* pin 1: the first CPUs of the mask; pin 2: the last ones (away
		 * from CPU 0 of the mask, where the HIP runtime's threads of the
		 * calling process tend to run) */
		if (pin == 2) {
			for (int c = CPU_SETSIZE - 1; c >= 0 && ncpu < threads; c--)
				if (CPU_ISSET(c, &mask))
					cpus[ncpu++] = c;
		} else {
			for (int c = 0; c < CPU_SETSIZE && ncpu < threads; c++)
				if (CPU_ISSET(c, &mask))
					cpus[ncpu++] = c;
		}
	}
	struct timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (int t = 0; t < threads; t++) {
		args[t].umem = umem;
		args[t].descs = descs;
		args[t].lo = (uint32_t)((uint64_t)n * t / threads);
		args[t].hi = (uint32_t)((uint64_t)n * (t + 1) / threads);
		args[t].o = o;
		args[t].verdicts = verdicts;
		args[t].cpu = (pin && t < ncpu) ? cpus[t] : -1;
		args[t].reps = reps;
		if (pthread_create(&tid[t], NULL, worker, &args[t]))
			return -1.0;
	}
	for (int t = 0; t < threads; t++)
		pthread_join(tid[t], NULL);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

/* ---- the callback as the reference app links it ---------------------
 * xsknf_packet_processor(pkt, len, ingress) with the options in globals, as
 * checksummer_user.c:24-28 keeps them: lets the AF_XDP runtime
 * (include/xsknf.h, xsknf_set_packet_processor) run the reference per-frame
 * path for config 1 (checksummer over veth, CPU only) and the runtime tests. */
static struct oracle_opts nf_opts = {1, 0, 1, 0};

void oracle_nf_set_options(int32_t csum_iterations, int32_t action, uint32_t num_interfaces)
{
	nf_opts.csum_iterations = csum_iterations;
	nf_opts.action = action;
	nf_opts.num_interfaces = num_interfaces;
}

int oracle_nf_packet_processor(void *pkt, unsigned len, unsigned ingress_ifindex)
{
	return oracle_packet_processor(pkt, len, ingress_ifindex, &nf_opts);
}

/* ---- the same NF as a two-phase batch hook (runtime tests) ----------
 * xsknf_batch_submit_fn / xsknf_batch_complete_fn for the runtime's
 * xsknf_set_batch_processor_async: submit only records the batch; complete
 * runs the per-frame oracle over every recorded batch up to its ticket.  So a
 * runtime that touched a batch's frames, descriptors or verdicts before its
 * complete would route frames on unset verdicts, and the tests see it.
 * oracle_nf_async_stats() counts submits made while another batch of the
 * worker was still recorded (the overlap the two-phase hook exists for). */
#define ORACLE_ASYNC_DEPTH 9   /* XSKNF_MAX_HOOK_DEPTH out + the one being submitted */
#define ORACLE_ASYNC_WORKERS 64

struct oracle_async_batch {
	uint8_t *umem;
	const struct oracle_desc *descs;
	uint32_t n;
	uint32_t ingress;
	int32_t *verdicts;
	uint64_t ticket;
};

static struct {
	struct oracle_async_batch q[ORACLE_ASYNC_DEPTH];
	unsigned head, count;
	uint64_t next;
	uint64_t submits, overlapped;
} oracle_async[ORACLE_ASYNC_WORKERS];

int oracle_nf_batch_submit(void *user, unsigned worker, void *umem, uint64_t umem_size,
		const struct oracle_desc *descs, uint32_t n, unsigned ingress, int32_t *verdicts,
		uint64_t *ticket)
{
	(void)user;
	(void)umem_size;
	if (worker >= ORACLE_ASYNC_WORKERS || !ticket)
		return -22;
	typeof(oracle_async[0]) *a = &oracle_async[worker];
	if (a->count == ORACLE_ASYNC_DEPTH)
		return -16;
	a->submits++;
	if (a->count)
		a->overlapped++;
	struct oracle_async_batch *b = &a->q[(a->head + a->count++) % ORACLE_ASYNC_DEPTH];
	*b = (struct oracle_async_batch){umem, descs, n, ingress, verdicts, ++a->next};
	for (uint32_t i = 0; i < n; i++)
		verdicts[i] = 0x7eadbeef;    /* "not computed yet" */
	*ticket = b->ticket;
	return 0;
}

int oracle_nf_batch_complete(void *user, unsigned worker, void *umem, uint64_t ticket)
{
	(void)user;
	(void)umem;
	if (worker >= ORACLE_ASYNC_WORKERS)
		return -22;
	typeof(oracle_async[0]) *a = &oracle_async[worker];
	while (a->count && a->q[a->head].ticket <= ticket) {
		const struct oracle_async_batch *b = &a->q[a->head];
		for (uint32_t i = 0; i < b->n; i++)
			b->verdicts[i] = oracle_packet_processor(b->umem + umem_offset(b->descs[i].addr),
					b->descs[i].len, b->ingress, &nf_opts);
		a->head = (a->head + 1) % ORACLE_ASYNC_DEPTH;
		a->count--;
	}
	return 0;
}

void oracle_nf_async_stats(unsigned worker, uint64_t *submits, uint64_t *overlapped)
{
	if (worker >= ORACLE_ASYNC_WORKERS)
		return;
	*submits = oracle_async[worker].submits;
	*overlapped = oracle_async[worker].overlapped;
}

void oracle_nf_async_reset(void)
{
	memset(oracle_async, 0, sizeof(oracle_async));
}

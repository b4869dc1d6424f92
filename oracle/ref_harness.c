/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY: drives the REFERENCE's own
 * xsknf_packet_processor(), compiled here from its verbatim text.
 *
 * oracle/ref_extract.sh copies the reference's lines (checksummer_user.c:15-18,
 * 24-25,28,30-112 and the declarations it needs from src/xsknf.h) into
 * oracle/_ref/checksummer_ref.c; this file #includes that text, so the
 * reference's static globals (opt_action :24, opt_csum_iterations :25) and
 * its `config` (:28) are set here exactly as the app's main() and
 * parse_command_line() set them (:144-161, :194), and calls the function as
 * process_batch_1if() does (src/xsknf.c:654-672, batch 64, with libxdp's
 * xsk_umem__add_offset_to_addr() translation at :659).  The result is
 * oracle/_ref/libcsum_ref.so (git-ignored).  Only tests/, tests/golden/ and
 * bench.py's cpu_baseline leg load it.
 */
#define _GNU_SOURCE
#include "checksummer_ref.c"

#include <pthread.h>
#include <sched.h>
#include <string.h>
#include <time.h>

struct ref_desc {               /* struct xdp_desc, linux/if_xdp.h */
	uint64_t addr;
	uint32_t len;
	uint32_t options;
};

/* -c REDIRECT|DROP, -i N (checksummer_user.c:149-161) and the library's
 * interface count (config.num_interfaces, filled by xsknf_parse_args) */
void ref_set_options(int csum_iterations, int action, unsigned num_interfaces)
{
	opt_csum_iterations = csum_iterations;
	opt_action = action == 0 ? ACTION_REDIRECT : ACTION_DROP;
	config.num_interfaces = num_interfaces;
}

int ref_packet_processor(void *pkt, unsigned len, unsigned ingress_ifindex)
{
	return xsknf_packet_processor(pkt, len, ingress_ifindex);
}

static inline uint64_t umem_offset(uint64_t addr)
{
	return (addr & ((1ULL << 48) - 1)) + (addr >> 48);
}

void ref_process_batch(uint8_t *umem, const struct ref_desc *descs, uint32_t n,
		uint32_t ingress, int32_t *verdicts, uint32_t batch)
{
	if (batch == 0)
		batch = 64;
	for (uint32_t b = 0; b < n; b += batch) {
		uint32_t rcvd = n - b < batch ? n - b : batch;
		for (uint32_t i = 0; i < rcvd; i++) {
			const struct ref_desc *d = &descs[b + i];
			verdicts[b + i] = xsknf_packet_processor(umem + umem_offset(d->addr),
					d->len, ingress);
		}
	}
}

/* ---- CPU baseline timing (bench.py cpu_baseline, kind "reference") ---- */

struct ref_worker {
	uint8_t *umem;
	const struct ref_desc *descs;
	uint32_t lo, hi;
	int32_t *verdicts;
	int cpu, reps;
};

static void *ref_worker_main(void *p)
{
	struct ref_worker *a = p;
	if (a->cpu >= 0) {
		cpu_set_t set;
		CPU_ZERO(&set);
		CPU_SET(a->cpu, &set);
		pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
	}
	for (int r = 0; r < a->reps; r++)
		ref_process_batch(a->umem, a->descs + a->lo, a->hi - a->lo, 0,
				a->verdicts + a->lo, 64);
	return NULL;
}

/* `reps` passes over n frames split contiguously over `threads` pthreads
 * (pinned to the first CPUs of the affinity mask when pin == 1, the last
 * ones when pin == 2); the options
 * are whatever ref_set_options() last set.  Wall seconds, or -1. */
double ref_time_batch(uint8_t *umem, const struct ref_desc *descs, uint32_t n,
		int32_t *verdicts, int threads, int reps, int pin)
{
	if (threads < 1 || threads > 1024)
		return -1.0;
	pthread_t tid[threads];
	struct ref_worker args[threads];
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
		args[t] = (struct ref_worker){umem, descs,
			(uint32_t)((uint64_t)n * t / threads),
			(uint32_t)((uint64_t)n * (t + 1) / threads),
			verdicts, (pin && t < ncpu) ? cpus[t] : -1, reps};
		if (pthread_create(&tid[t], NULL, ref_worker_main, &args[t]))
			return -1.0;
	}
	for (int t = 0; t < threads; t++)
		pthread_join(tid[t], NULL);
	clock_gettime(CLOCK_MONOTONIC, &t1);
	return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
}

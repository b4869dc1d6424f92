// hook_bench.c -- frames per second through the whole NF worker loop
// (libxsknf's worker on an emulated queue, src/xsknf.c:716-742 in shape) with
// the checksummer as
//   cpu    the reference per-frame NF on one worker core: the reference's own
//          xsknf_packet_processor() compiled from its verbatim lines
//          (oracle/_ref/libcsum_ref.so, loaded at run time) where that library
//          was built, else the CPU restatement ("cpu_nf" in the output says which),
//   sync   the GPU hook, one batch at a time (xsknf_gpu_hook_process),
//   async  the GPU hook, two-phase (xsknf_gpu_hook_submit / _complete: the
//          worker receives batch k+1 while the GPU checksums batch k),
//   null   an NF that forwards without touching the frame (the harness's own
//          ceiling: this thread's deliver / transmit copies and the rings).
// This thread plays the kernel: it keeps the rx ring fed with LEN-byte
// Eth/IPv4/UDP frames and drains the tx ring, and counts what the worker
// received over SECONDS after a half-second warm-up.
//
//   hook_bench MODE LEN BATCH SECONDS [ZEROCOPY|STAGED|RESIDENT [DEPTH]]   (DEPTH: batches in flight, async)
//
// HOOK_BENCH_CHECKS=nic gives the frames the UDP checksums a NIC's offload
// writes (tests/gen-traffic.lua:120; RFC 768, fully folded), as the reference's
// traffic carries them: the GPU kernels then write nothing back for all but
// the carry-loss frames.  Default: random check bytes (every check changes).
//
// The feeding thread (this one) is pinned to the last CPU of the process's
// affinity set once the worker runs (the worker takes the first, as
// src/xsknf.c:1049-1095 pins workers), so the two never share a core;
// HOOK_BENCH_FEEDER_CPU=-1 leaves it unpinned.
//
// Prints one JSON line.  Tool, not product: it links the oracle only as the CPU
// NF of mode "cpu" (the reference path, as tools/config1.py does).
#define _GNU_SOURCE
#include <arpa/inet.h>
#include <dlfcn.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/xsknf.h"
#include "../include/xsknf_gpu.h"

void oracle_nf_set_options(int32_t csum_iterations, int32_t action, uint32_t num_interfaces);
int oracle_nf_packet_processor(void *pkt, unsigned len, unsigned ingress_ifindex);

// The reference's own per-packet function, if oracle/_ref was built (next to this binary's tree).
static xsknf_packet_processor_fn load_reference_nf(const char *argv0)
{
	char path[4096];
	const char *slash = strrchr(argv0, '/');
	const int dir = slash ? (int)(slash - argv0) : 1;
	snprintf(path, sizeof(path), "%.*s/../../oracle/_ref/libcsum_ref.so", dir, slash ? argv0 : ".");
	void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
	if (!h)
		return NULL;
	void (*set)(int, int, unsigned) = (void (*)(int, int, unsigned))dlsym(h, "ref_set_options");
	xsknf_packet_processor_fn fn = (xsknf_packet_processor_fn)dlsym(h, "xsknf_packet_processor");
	if (!set || !fn)
		return NULL;
	set(1, 0, 1);   // -i 1, -c REDIRECT, one interface: the options the GPU modes run with
	return fn;
}

static int null_nf(void *pkt, unsigned len, unsigned ingress)
{
	(void)pkt;
	(void)len;
	(void)ingress;
	return 0;
}

// RFC 768 UDP checksum of an Eth/IPv4 (ihl 5)/UDP frame, as a NIC's offload fills it in
static uint16_t nic_udp_check(const uint8_t *f, unsigned len)
{
	uint64_t s = 17 + ((unsigned)f[38] << 8 | f[39]);
	for (unsigned i = 26; i < 34; i += 2)
		s += (unsigned)f[i] << 8 | f[i + 1];
	for (unsigned i = 34; i < len; i += 2)
		if (i != 40)
			s += (unsigned)f[i] << 8 | (i + 1 < len ? f[i + 1] : 0);
	while (s >> 16)
		s = (s & 0xffff) + (s >> 16);
	const uint16_t c = (uint16_t)~s;
	return c ? c : 0xffff;
}

static double now_s(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static uint64_t rx_count(void)
{
	struct xsknf_socket_stats s;
	return xsknf_get_socket_stats(0, 0, &s) ? 0 : s.rx_npkts;
}

int main(int argc, char **argv)
{
	if (argc < 5) {
		fprintf(stderr, "usage: %s cpu|sync|async|null LEN BATCH SECONDS [ZEROCOPY|STAGED]\n", argv[0]);
		return 2;
	}
	const char *mode = argv[1];
	const unsigned len = (unsigned)atoi(argv[2]);
	const unsigned batch = (unsigned)atoi(argv[3]);
	const double secs = atof(argv[4]);
	const int path = argc > 5 && !strcmp(argv[5], "STAGED")     ? XSKNF_GPU_PATH_STAGED
	                 : argc > 5 && !strcmp(argv[5], "RESIDENT") ? XSKNF_GPU_PATH_RESIDENT
	                                                            : XSKNF_GPU_PATH_ZEROCOPY;
	const unsigned depth = argc > 6 ? (unsigned)atoi(argv[6]) : 1;
	if (len < 42 || len > 3800 || batch == 0) {
		fprintf(stderr, "bad LEN / BATCH\n");
		return 2;
	}

	struct xsknf_config cfg;
	memset(&cfg, 0, sizeof(cfg));
	char n0[] = "emu0";
	cfg.interfaces[0] = n0;
	cfg.bind_flags[0] = 1u << 3;   // XDP_USE_NEED_WAKEUP
	cfg.num_interfaces = 1;
	cfg.workers = 1;
	cfg.working_mode = MODE_AF_XDP;
	cfg.xdp_flags = 1u | (1u << 2);
	cfg.batch_size = batch;
	cfg.xsk_frame_size = 4096;
	int rc = xsknf_init(&cfg, NULL);
	if (rc) {
		fprintf(stderr, "xsknf_init: %d\n", rc);
		return 1;
	}
	struct xsknf_gpu_hook *hook = NULL;
	const struct xsknf_csum_opts opts = {1, XSKNF_CSUM_ACTION_REDIRECT, 1, 0};
	const char *cpu_nf = "none";
	if (!strcmp(mode, "cpu")) {
		xsknf_packet_processor_fn ref = load_reference_nf(argv[0]);
		if (ref) {
			cpu_nf = "reference";
			xsknf_set_packet_processor(ref);
		} else {
			cpu_nf = "port";
			oracle_nf_set_options(1, 0, 1);
			xsknf_set_packet_processor(oracle_nf_packet_processor);
		}
	} else if (!strcmp(mode, "null")) {
		xsknf_set_packet_processor(null_nf);
	} else {
		rc = xsknf_gpu_hook_create(&hook, &opts, 1, path, batch, len);
		if (rc) {
			fprintf(stderr, "hook: %d (%s)\n", rc, xsknf_gpu_last_error());
			return 1;
		}
		if (!strcmp(mode, "sync"))
			xsknf_set_batch_processor((xsknf_batch_processor_fn)xsknf_gpu_hook_process, hook);
		else
			xsknf_set_batch_processor_async((xsknf_batch_submit_fn)xsknf_gpu_hook_submit,
					(xsknf_batch_complete_fn)xsknf_gpu_hook_complete, hook);
		if (xsknf_set_batch_depth(depth)) {
			fprintf(stderr, "bad DEPTH\n");
			return 2;
		}
	}

	// frames as tests/gen-traffic.lua builds them (Eth/IPv4 ihl 5/UDP, 256 flows)
	enum { BURST = 256, TXMAX = 1024, TXSTRIDE = 64 };
	const char *ck = getenv("HOOK_BENCH_CHECKS");
	const int nic = ck && !strcmp(ck, "nic");
	uint8_t *frames = calloc(BURST, len);
	uint32_t lens[BURST];
	uint64_t rng = 0x58534B4E;
	for (unsigned k = 0; k < BURST; k++) {
		uint8_t *f = frames + (size_t)k * len;
		for (unsigned i = 0; i < len; i++) {
			rng = rng * 6364136223846793005ull + 1442695040888963407ull;
			f[i] = (uint8_t)(rng >> 33);
		}
		f[12] = 0x08, f[13] = 0x00, f[14] = 0x45, f[15] = 0;
		const uint16_t tot = htons((uint16_t)(len - 14)), ulen = htons((uint16_t)(len - 34));
		memcpy(f + 16, &tot, 2);
		f[22] = 64, f[23] = 17;
		f[26] = 10, f[27] = 0, f[28] = 0, f[29] = (uint8_t)k;
		f[30] = 172, f[31] = 0, f[32] = 0, f[33] = 1;
		f[34] = 0x13, f[35] = 0x88, f[36] = 0, f[37] = 80;
		memcpy(f + 38, &ulen, 2);
		if (nic) {
			const uint16_t c = nic_udp_check(f, len);
			f[40] = (uint8_t)(c >> 8), f[41] = (uint8_t)c;
		}
		lens[k] = len;
	}
	uint8_t *txbuf = malloc((size_t)TXMAX * TXSTRIDE);
	uint32_t txlens[TXMAX];

	rc = xsknf_start_workers();
	if (rc) {
		fprintf(stderr, "start: %d\n", rc);
		return 1;
	}
	int feeder_cpu = -1;
	{
		const char *fc = getenv("HOOK_BENCH_FEEDER_CPU");
		cpu_set_t set;
		if ((!fc || atoi(fc) >= 0) && sched_getaffinity(0, sizeof(set), &set) == 0) {
			for (int c = CPU_SETSIZE - 1; c >= 0; c--)
				if (CPU_ISSET(c, &set)) {
					feeder_cpu = fc ? atoi(fc) : c;
					break;
				}
			CPU_ZERO(&set);
			CPU_SET(feeder_cpu, &set);
			if (pthread_setaffinity_np(pthread_self(), sizeof(set), &set))
				feeder_cpu = -1;
		}
	}
	const double t0 = now_s();
	double tm = 0;
	uint64_t rx0 = 0;
	for (;;) {
		const double t = now_s();
		if (!tm && t - t0 >= 0.5) {
			tm = t;
			rx0 = rx_count();
		}
		if (tm && t - tm >= secs)
			break;
		if (xsknf_emu_deliver(0, 0, frames, lens, BURST, len) < 0)
			break;
		xsknf_emu_transmit(0, 0, txbuf, txlens, TXMAX, TXSTRIDE);
		if (xsknf_worker_error(0))
			break;
	}
	const double t1 = now_s();
	const uint64_t rx = rx_count() - rx0;
	const int err = xsknf_worker_error(0);
	xsknf_stop_workers();
	if (hook)
		xsknf_gpu_hook_destroy(hook);
	xsknf_cleanup();
	const double mpps = rx / (t1 - tm) / 1e6;
	printf("{\"checks\": \"%s\", \"mode\": \"%s\", \"len\": %u, \"batch\": %u, \"path\": \"%s\", \"depth\": %u, "
	       "\"seconds\": %.2f, \"mpps\": %.3f, \"gbps\": %.2f, \"feeder_cpu\": %d, \"cpu_nf\": \"%s\", "
	       "\"worker_error\": %d}\n",
	       nic ? "nic" : "random", mode, len, batch,
	       path == XSKNF_GPU_PATH_STAGED ? "STAGED" : path == XSKNF_GPU_PATH_RESIDENT ? "RESIDENT" : "ZEROCOPY",
	       depth, t1 - tm, mpps,
	       mpps * len / 1e3, feeder_cpu, cpu_nf, err);
	free(frames);
	free(txbuf);
	return err ? 1 : 0;
}

// san_runtime.c -- the host runtime under ThreadSanitizer / AddressSanitizer
// (TSAN/ASAN runs of the host C).  Test infrastructure: built and
// run by tests/test_sanitizers.py with gcc -fsanitize=...
//
// Two workers x two emulated interfaces ("emu0", "emu1": in-memory rings with
// the kernel's semantics, include/xsknf.h), the reference per-frame NF (the
// CPU oracle; REDIRECT: a frame leaves on (ingress + 1) % 2, or `drop`), frames delivered
// and collected by this thread while the workers run: every frame the oracle
// forwards must come out once, on the oracle's interface, byte for byte as the
// oracle rewrites it; the rest must be dropped.  The worker threads, the
// multi-interface path (process_batch / complete_tx, cross-UMEM copies) and
// the stats reads from this thread are what the sanitizers watch.
#include <arpa/inet.h>
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../include/xsknf.h"

struct oracle_opts {
	int32_t csum_iterations;
	int32_t action;
	uint32_t num_interfaces;
	uint32_t reserved;
};
int oracle_packet_processor(void *pkt, unsigned len, unsigned ingress_ifindex, const struct oracle_opts *o);
void oracle_nf_set_options(int32_t csum_iterations, int32_t action, uint32_t num_interfaces);
int oracle_nf_packet_processor(void *pkt, unsigned len, unsigned ingress_ifindex);
/* the same NF as a two-phase hook (argv[2] == "async": one batch in flight per worker) */
int oracle_nf_batch_submit(void *user, unsigned worker, void *umem, uint64_t umem_size,
		const struct xdp_desc *descs, uint32_t n, unsigned ingress, int32_t *verdicts, uint64_t *ticket);
int oracle_nf_batch_complete(void *user, unsigned worker, void *umem, uint64_t ticket);

#define WORKERS 2
#define IFACES 2
#define NFRAMES 3000          /* per (worker, iface) queue */
#define STRIDE 1600

static uint64_t rng = 0x58534B4E;
static uint32_t next_rand(void)
{
	rng = rng * 6364136223846793005ull + 1442695040888963407ull;
	return (uint32_t)(rng >> 33);
}

/* Eth / IPv4 / UDP with a 32-bit tag (frame id) in its last 4 bytes; a few frames
 * take the reference's other branches (not IPv4, not UDP, odd ihl) */
static uint32_t build(uint8_t *f, uint32_t id)
{
	const uint32_t len = 60 + next_rand() % 1400;
	for (uint32_t i = 0; i < len; i++)
		f[i] = (uint8_t)next_rand();
	const uint32_t kind = next_rand() % 20;
	f[12] = 0x08;
	f[13] = kind == 0 ? 0xdd : 0x00;                  /* 1 in 20: not IPv4 */
	f[14] = kind == 1 ? 0x46 : 0x45;                  /* 1 in 20: ihl 6 */
	uint16_t tot = htons((uint16_t)(len - 14));
	memcpy(f + 16, &tot, 2);
	f[23] = kind == 2 ? 6 : 17;                       /* 1 in 20: TCP */
	const uint32_t u = 14 + 4 * (f[14] & 15);
	uint16_t ulen = htons((uint16_t)(len - u));
	memcpy(f + u + 4, &ulen, 2);
	f[u + 6] = f[u + 7] = 0;
	memcpy(f + len - 4, &id, 4);                           /* the tag: last 4 bytes */
	return len;
}

static uint8_t *orig[WORKERS][IFACES];
static uint32_t lens[WORKERS][IFACES][NFRAMES];

int main(int argc, char **argv)
{
	const int32_t action = argc > 1 && !strcmp(argv[1], "drop");   /* 0 REDIRECT, 1 DROP */
	struct xsknf_config cfg;
	memset(&cfg, 0, sizeof(cfg));
	char n0[] = "emu0", n1[] = "emu1";
	cfg.interfaces[0] = n0;
	cfg.interfaces[1] = n1;
	cfg.bind_flags[0] = cfg.bind_flags[1] = 1u << 3;   /* XDP_USE_NEED_WAKEUP */
	cfg.num_interfaces = IFACES;
	cfg.workers = WORKERS;
	cfg.working_mode = MODE_AF_XDP;
	cfg.xdp_flags = 1u | (1u << 2);
	cfg.batch_size = 64;
	cfg.xsk_frame_size = 4096;

	int rc = xsknf_init(&cfg, NULL);
	if (rc) {
		fprintf(stderr, "xsknf_init: %d\n", rc);
		return 2;
	}
	oracle_nf_set_options(1, action, IFACES);
	if (argc > 2 && !strcmp(argv[2], "async"))
		xsknf_set_batch_processor_async(oracle_nf_batch_submit, oracle_nf_batch_complete, NULL);
	else
		xsknf_set_packet_processor(oracle_nf_packet_processor);
	for (int w = 0; w < WORKERS; w++)
		for (int i = 0; i < IFACES; i++) {
			orig[w][i] = malloc((size_t)NFRAMES * STRIDE);
			for (uint32_t k = 0; k < NFRAMES; k++) {
				const uint32_t id = ((uint32_t)w << 24) | ((uint32_t)i << 20) | k;
				lens[w][i][k] = build(orig[w][i] + (size_t)k * STRIDE, id);
			}
		}
	rc = xsknf_start_workers();
	if (rc) {
		fprintf(stderr, "xsknf_start_workers: %d\n", rc);
		return 2;
	}

	/* what must come out: oracle on a copy of each frame */
	const struct oracle_opts o = {1, action, IFACES, 0};
	long expect_tx = 0, got_tx = 0, bad = 0;
	uint8_t *seen = calloc((size_t)WORKERS * IFACES * NFRAMES, 1);
	uint32_t sent[WORKERS][IFACES] = {{0}};
	uint8_t *out = malloc((size_t)512 * STRIDE);
	uint32_t olens[512];
	uint8_t frame[STRIDE];
	for (int w = 0; w < WORKERS; w++)
		for (int i = 0; i < IFACES; i++)
			for (uint32_t k = 0; k < NFRAMES; k++) {
				memcpy(frame, orig[w][i] + (size_t)k * STRIDE, lens[w][i][k]);
				if (oracle_packet_processor(frame, lens[w][i][k], (unsigned)i, &o) >= 0)
					expect_tx++;
			}

	const time_t t_end = time(NULL) + 60;
	long quiet = 0;
	while (time(NULL) < t_end) {
		int progress = 0, all_sent = 1;
		for (int w = 0; w < WORKERS; w++)
			for (int i = 0; i < IFACES; i++) {
				if (sent[w][i] < NFRAMES) {
					const uint32_t n = NFRAMES - sent[w][i] < 256 ? NFRAMES - sent[w][i] : 256;
					rc = xsknf_emu_deliver(w, i, orig[w][i] + (size_t)sent[w][i] * STRIDE,
							       lens[w][i] + sent[w][i], n, STRIDE);
					if (rc < 0) {
						fprintf(stderr, "deliver: %d\n", rc);
						return 2;
					}
					sent[w][i] += rc;
					progress |= rc > 0;
					all_sent &= sent[w][i] == NFRAMES;
				}
				const int m = xsknf_emu_transmit(w, i, out, olens, 512, STRIDE);
				for (int j = 0; j < m; j++) {
					const uint8_t *p = out + (size_t)j * STRIDE;
					uint32_t id;
					memcpy(&id, p + olens[j] - 4, 4);
					const uint32_t sw = id >> 24, si = (id >> 20) & 15, sk = id & 0xfffff;
					const size_t slot = ((size_t)sw * IFACES + si) * NFRAMES + sk;
					if (sw >= WORKERS || si >= IFACES || sk >= NFRAMES || seen[slot] ||
					    olens[j] != lens[sw][si][sk]) {
						bad++;
						continue;
					}
					seen[slot] = 1;
					memcpy(frame, orig[sw][si] + (size_t)sk * STRIDE, olens[j]);
					const int v = oracle_packet_processor(frame, olens[j], si, &o);
					if (v != i || w != (int)sw || memcmp(frame, p, olens[j]))
						bad++;
				}
				got_tx += m;
				progress |= m > 0;
				if (xsknf_worker_error(w)) {
					fprintf(stderr, "worker %d error %d\n", w, xsknf_worker_error(w));
					return 2;
				}
			}
		/* stats read while the workers run (the reference's stats thread) */
		struct xsknf_socket_stats st;
		unsigned long rx = 0;
		for (int w = 0; w < WORKERS; w++)
			for (int i = 0; i < IFACES; i++)
				if (!xsknf_get_socket_stats(w, i, &st))
					rx += st.rx_npkts;
		if (all_sent && got_tx >= expect_tx && rx == (unsigned long)WORKERS * IFACES * NFRAMES) {
			if (!progress && ++quiet > 200)
				break;
		} else {
			quiet = 0;
		}
		usleep(200);
	}
	xsknf_stop_workers();
	xsknf_cleanup();
	printf("expected tx %ld, got %ld, bad %ld\n", expect_tx, got_tx, bad);
	for (int w = 0; w < WORKERS; w++)
		for (int i = 0; i < IFACES; i++)
			free(orig[w][i]);
	free(seen);
	free(out);
	return (bad == 0 && got_tx == expect_tx) ? 0 : 1;
}

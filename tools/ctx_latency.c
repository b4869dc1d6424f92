// ctx_latency.c -- where a small host-path batch's time goes: CPU time inside
// xsknf_gpu_ctx_submit (descriptor copy, launch, event) and inside
// xsknf_gpu_ctx_wait, for batches of N frames of LEN bytes in a pinned UMEM,
// DEPTH - 1 batches in flight behind the one being submitted (default 2, at most 8; 1 =
// each batch waited for right after its submit: the round trip itself).
//   ctx_latency LEN N ITERS [ZEROCOPY|STAGED|RESIDENT [DEPTH]]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/xsknf_gpu.h"

static double now_us(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

int main(int argc, char **argv)
{
	if (argc < 4)
		return 2;
	const unsigned len = (unsigned)atoi(argv[1]), n = (unsigned)atoi(argv[2]), iters = (unsigned)atoi(argv[3]);
	const int path = argc > 4 && !strcmp(argv[4], "STAGED")     ? XSKNF_GPU_PATH_STAGED
	                 : argc > 4 && !strcmp(argv[4], "RESIDENT") ? XSKNF_GPU_PATH_RESIDENT
	                                                            : XSKNF_GPU_PATH_ZEROCOPY;
	const unsigned depth = argc > 5 ? (unsigned)atoi(argv[5]) : 2;
	if (depth < 1 || depth > 8)
		return 2;
	const unsigned nb = 64;   // distinct batches cycled through
	const size_t chunk = 2048, size = (size_t)nb * n * chunk;
	uint8_t *umem = aligned_alloc(4096, size);
	memset(umem, 0x5a, size);
	struct xsknf_gpu_desc *d = malloc(sizeof(*d) * (size_t)nb * n);
	for (size_t i = 0; i < (size_t)nb * n; i++) {
		uint8_t *f = umem + i * chunk + 256;
		f[12] = 8, f[13] = 0, f[14] = 0x45, f[23] = 17;
		d[i].addr = i * chunk + 256;
		d[i].len = len;
		d[i].options = 0;
	}
	int32_t *v = malloc(sizeof(int32_t) * (size_t)nb * n);
	struct xsknf_gpu_ctx *c;
	const struct xsknf_csum_opts o = {1, XSKNF_CSUM_ACTION_REDIRECT, 1, 0};
	if (xsknf_gpu_ctx_create(&c, 0, path, n, len) || xsknf_gpu_ctx_register_umem(c, umem, size)) {
		fprintf(stderr, "ctx: %s\n", xsknf_gpu_last_error());
		return 1;
	}
	double t_sub = 0, t_wait = 0;
	uint64_t tk[8] = {0};
	const double t0 = now_us();
	for (unsigned i = 0; i < iters; i++) {
		const unsigned b = i % nb;
		double a = now_us();
		if (xsknf_gpu_ctx_submit(c, d + (size_t)b * n, n, 0, &o, v + (size_t)b * n, &tk[i % 8]))
			return 1;
		double m = now_us();
		if (i + 1 >= depth && xsknf_gpu_ctx_wait(c, tk[(i + 1 - depth) % 8]))
			return 1;
		double e = now_us();
		if (i >= 16) {
			t_sub += m - a;
			t_wait += e - m;
		}
	}
	xsknf_gpu_ctx_wait(c, tk[(iters - 1) % 8]);
	const double total = now_us() - t0;
	const unsigned k = iters - 16;
	printf("{\"len\": %u, \"n\": %u, \"path\": \"%s\", \"depth\": %u, \"us_per_batch\": %.2f, "
	       "\"submit_cpu_us\": %.2f, \"wait_us\": %.2f}\n", len, n,
	       path == XSKNF_GPU_PATH_STAGED ? "STAGED" : path == XSKNF_GPU_PATH_RESIDENT ? "RESIDENT" : "ZEROCOPY", depth,
	       total / iters, t_sub / k, t_wait / k);
	xsknf_gpu_ctx_destroy(c);
	return 0;
}

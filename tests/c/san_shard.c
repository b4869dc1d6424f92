/*
 * san_shard.c -- the multi-device path's host arithmetic (xsknf_amd/csrc/
 * shard_plan.cpp: xsknf_gpu_shard_plan / _rebase / _pack_plan) under
 * AddressSanitizer + UBSan, on random and edge-case descriptor sets: empty
 * batches, more shards than frames, zero and huge lengths, unaligned-mode
 * addresses, descriptors outside the UMEM, a UMEM of 0 bytes.  Checks the
 * invariants every caller relies on; prints "ok <cases>".  CPU only
 * (tests/test_sanitizers.py builds and runs it).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "xsknf_gpu.h"

#define OUT_OF_RANGE (1ULL << 47)

static uint64_t st = 0x9E3779B97F4A7C15ULL;
static uint64_t rnd(void)
{
	st ^= st >> 12;
	st ^= st << 25;
	st ^= st >> 27;
	return st * 0x2545F4914F6CDD1DULL;
}

static uint64_t off_of(uint64_t a)
{
	return (a & XSKNF_GPU_UNALIGNED_BUF_ADDR_MASK) + (a >> XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT);
}

static int inside(const struct xsknf_gpu_desc *d, uint64_t size)
{
	const uint64_t o = off_of(d->addr);
	return o <= size && d->len <= size - o;
}

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "case %d: %s failed (line %d)\n", cs, #c, __LINE__); return 1; } } while (0)

int main(void)
{
	int cs;
	for (cs = 0; cs < 3000; cs++) {
		const uint64_t n = cs % 7 == 0 ? 0 : rnd() % (cs % 5 == 0 ? 5 : 3000);
		const uint32_t k = 1 + (uint32_t)(rnd() % (cs % 3 == 0 ? 70 : 9));
		const uint64_t size = cs % 11 == 0 ? 0 : 1 + rnd() % (1ULL << (10 + cs % 25));
		struct xsknf_gpu_desc *d = malloc(sizeof(*d) * (n ? n : 1));
		struct xsknf_gpu_desc *r = malloc(sizeof(*r) * (n ? n : 1));
		struct xsknf_gpu_desc *p = malloc(sizeof(*p) * (n ? n : 1));
		uint64_t *b = malloc(sizeof(uint64_t) * (k + 1)), *sp = malloc(sizeof(uint64_t) * 2 * k);
		uint64_t *sz = malloc(sizeof(uint64_t) * k);
		for (uint64_t i = 0; i < n; i++) {
			const uint64_t kind = rnd() % 16;
			d[i].len = kind == 0 ? 0 : kind == 1 ? 0xFFFFFFFFu : (uint32_t)(rnd() % 9100);
			d[i].options = (uint32_t)rnd();
			uint64_t o = size ? rnd() % size : 0;
			if (kind == 2)
				o = size + rnd() % 4096;                   /* past the UMEM */
			if (kind == 3 || kind == 4)                        /* unaligned mode: base | offset << 48 */
				d[i].addr = (o & ~255ULL) | ((o & 255ULL) << XSKNF_GPU_UNALIGNED_BUF_OFFSET_SHIFT);
			else
				d[i].addr = o;
			if (kind == 5)
				d[i].addr = rnd();                         /* anything */
		}
		CHECK(xsknf_gpu_shard_plan(d, n, size, k, b, sp) == 0);
		CHECK(b[0] == 0 && b[k] == n);
		for (uint32_t s = 0; s < k; s++) {
			CHECK(b[s] <= b[s + 1]);
			CHECK(sp[2 * s] <= sp[2 * s + 1] && sp[2 * s + 1] <= size);
			for (uint64_t i = b[s]; i < b[s + 1]; i++)
				if (inside(&d[i], size))
					CHECK(off_of(d[i].addr) >= sp[2 * s] && off_of(d[i].addr) + d[i].len <= sp[2 * s + 1]);
			CHECK(xsknf_gpu_shard_rebase(d + b[s], b[s + 1] - b[s], sp[2 * s], size, r + b[s]) == 0);
			for (uint64_t i = b[s]; i < b[s + 1]; i++) {
				CHECK(r[i].len == d[i].len && r[i].options == d[i].options);
				if (inside(&d[i], size))
					CHECK(r[i].addr + r[i].len <= sp[2 * s + 1] - sp[2 * s]);
				else
					CHECK(r[i].addr == OUT_OF_RANGE);
			}
		}
		const uint64_t base = (rnd() & ~0xFFFULL & ((1ULL << 47) - 1)) | (rnd() & 15);
		CHECK(xsknf_gpu_shard_pack_plan(d, n, base, size, k, b, p, sz) == 0);
		for (uint32_t s = 0; s < k; s++) {
			uint64_t end = 0;
			for (uint64_t i = b[s]; i < b[s + 1]; i++) {
				CHECK(p[i].len == d[i].len && p[i].options == d[i].options);
				if (!inside(&d[i], size)) {
					CHECK(p[i].addr == OUT_OF_RANGE);
					continue;
				}
				if (!p[i].len)
					continue;                                  /* no bytes: no slot (verdict -1 either way) */
				CHECK(p[i].addr % 16 == (base + off_of(d[i].addr)) % 16);
				CHECK(p[i].addr + p[i].len <= sz[s]);
				CHECK(p[i].addr >= end);                           /* in order, no overlap */
				end = p[i].addr + p[i].len;
			}
		}
		/* bad arguments are refused, not dereferenced */
		CHECK(xsknf_gpu_shard_plan(d, n, size, 0, b, sp) < 0);
		CHECK(n == 0 || xsknf_gpu_shard_plan(NULL, n, size, k, b, sp) < 0);
		b[k] = n + 1;
		CHECK(xsknf_gpu_shard_pack_plan(d, n, base, size, k, b, p, sz) < 0);
		free(d); free(r); free(p); free(b); free(sp); free(sz);
	}
	printf("ok %d\n", cs);
	return 0;
}

// xsk_ring.h -- single-producer / single-consumer views of the AF_XDP rings.
//
// The kernel shares each ring as {u32 producer, u32 consumer, u32 flags,
// entries[size]} (linux/if_xdp.h struct xdp_ring_offset); the side that owns
// an index writes it with release order after filling / draining entries and
// the other side reads it with acquire order.  Each view caches the peer's
// index so that most reserve/peek calls touch no shared cache line.
// Emulated queues (xsknf.h "emu<k>") use the same views on heap memory.
#ifndef XSKNF_AMD_XSK_RING_H
#define XSKNF_AMD_XSK_RING_H

#include <linux/if_xdp.h>
#include <stdint.h>

struct xsk_ring {
	uint32_t *producer;
	uint32_t *consumer;
	uint32_t *flags;
	void *entries;
	uint32_t size;          // power of two
	uint32_t mask;
	uint32_t local;         // own index: next slot to fill (producer) / read (consumer)
	uint32_t peer;          // cached peer index (producer views keep consumer + size)
};

static inline uint32_t ring_load(const uint32_t *p)
{
	return __atomic_load_n(p, __ATOMIC_ACQUIRE);
}

static inline void ring_store(uint32_t *p, uint32_t v)
{
	__atomic_store_n(p, v, __ATOMIC_RELEASE);
}

/* ---- producer side (fill, tx; rx and completion on emulated queues) ---- */

static inline void ring_prod_init(struct xsk_ring *r)
{
	r->local = ring_load(r->producer);
	r->peer = ring_load(r->consumer) + r->size;
}

static inline uint32_t ring_prod_space(struct xsk_ring *r, uint32_t want)
{
	uint32_t space = r->peer - r->local;
	if (space < want) {
		r->peer = ring_load(r->consumer) + r->size;
		space = r->peer - r->local;
	}
	return space;
}

// all-or-nothing, like the reference's use of xsk_ring_prod__reserve()
static inline uint32_t ring_reserve(struct xsk_ring *r, uint32_t n, uint32_t *idx)
{
	if (ring_prod_space(r, n) < n)
		return 0;
	*idx = r->local;
	r->local += n;
	return n;
}

static inline void ring_submit(struct xsk_ring *r, uint32_t n)
{
	ring_store(r->producer, ring_load(r->producer) + n);
}

/* ---- consumer side (rx, completion; fill and tx on emulated queues) ---- */

static inline void ring_cons_init(struct xsk_ring *r)
{
	r->local = ring_load(r->consumer);
	r->peer = ring_load(r->producer);
}

static inline uint32_t ring_peek(struct xsk_ring *r, uint32_t max, uint32_t *idx)
{
	uint32_t avail = r->peer - r->local;
	if (avail == 0) {
		r->peer = ring_load(r->producer);
		avail = r->peer - r->local;
	}
	if (avail > max)
		avail = max;
	if (avail) {
		*idx = r->local;
		r->local += avail;
	}
	return avail;
}

static inline void ring_release(struct xsk_ring *r, uint32_t n)
{
	ring_store(r->consumer, ring_load(r->consumer) + n);
}

static inline int ring_needs_wakeup(const struct xsk_ring *r)
{
	return r->flags && (__atomic_load_n(r->flags, __ATOMIC_RELAXED) & XDP_RING_NEED_WAKEUP);
}

static inline struct xdp_desc *ring_desc(struct xsk_ring *r, uint32_t idx)
{
	return &((struct xdp_desc *)r->entries)[idx & r->mask];
}

static inline uint64_t *ring_addr(struct xsk_ring *r, uint32_t idx)
{
	return &((uint64_t *)r->entries)[idx & r->mask];
}

#endif

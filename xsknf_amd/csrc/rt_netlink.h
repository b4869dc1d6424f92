// rt_netlink.h -- rtnetlink helpers of the AF_XDP runtime (internal).
#ifndef XSKNF_AMD_RT_NETLINK_H
#define XSKNF_AMD_RT_NETLINK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// attach prog_fd as the XDP program of ifindex (prog_fd < 0 detaches);
// xdp_flags are the XDP_FLAGS_* of linux/if_link.h.  0 or -errno.
int xsknf_nl_set_xdp(int ifindex, int prog_fd, uint32_t xdp_flags);
// create the veth pair name <-> peer in the current network namespace
int xsknf_nl_create_veth(const char *name, const char *peer);
int xsknf_nl_link_up(int ifindex);

#ifdef __cplusplus
}
#endif

#endif

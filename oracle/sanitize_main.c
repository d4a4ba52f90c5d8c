/* oracle/sanitize_main.c — TEST INFRASTRUCTURE ONLY (sanitizer build of the CPU
 * restatement). Runs every oracle entry point over fuzz frames held in heap buffers of exactly
 * the size each contract allows (len bytes; cap bytes for a VLAN edit), built with
 * -fsanitize=address,undefined by `make -C oracle sanitize`: any read or write past a frame, or
 * undefined arithmetic, aborts the run. Usage: nfo_sanitize [frames] [seed] */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nfcs_oracle.h"

int main(int argc, char** argv) {
    const unsigned long n = argc > 1 ? strtoul(argv[1], NULL, 10) : 20000;
    const unsigned long long seed = argc > 2 ? strtoull(argv[2], NULL, 10) : 4242;
    static uint8_t tmp[9016];
    unsigned long long acc = 0;
    for (unsigned long i = 0; i < n; ++i) {
        const uint32_t len = nfo_fuzz_frame(seed, i, tmp);
        /* update_checksums: exactly len bytes */
        uint8_t* f = (uint8_t*)malloc(len ? len : 1);
        memcpy(f, tmp, len);
        acc += (unsigned)nfo_update(f, len);
        /* L3 forward with a next hop and without one */
        static const uint8_t nh[12] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12};
        memcpy(f, tmp, len);
        acc += (unsigned)nfo_l3_forward(f, len, (i & 1) ? nh : NULL);
        /* flow key */
        uint8_t rec[64];
        acc += nfo_flow_key(tmp, len, rec) ^ rec[0];
        free(f);
        /* VLAN push (buffer of len + 4 bytes) and pop (len bytes) */
        const uint32_t caps[2] = {len + 4, len};
        const uint32_t ops[2] = {NFO_VLAN_PUSH | (3u << 13) | (uint32_t)(i & 0xFFF), NFO_VLAN_POP};
        for (int k = 0; k < 2; ++k) {
            uint8_t* g = (uint8_t*)malloc(caps[k] ? caps[k] : 1);
            memset(g, 0, caps[k]);
            memcpy(g, tmp, len);
            uint32_t l = len;
            acc += (unsigned)nfo_vlan(g, &l, caps[k], ops[k]) + l;
            free(g);
        }
    }
    printf("sanitize_frames=%lu acc=%llu\n", n, acc);
    return 0;
}

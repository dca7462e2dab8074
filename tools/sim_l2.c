/* Set-associative LRU cache model for tools/sim_l2.py (a design probe, not product code):
 * counts the misses of a stream of 128-B line ids through one XCD's L2 (sets x ways). */
#include <stdint.h>
#include <stdlib.h>

int64_t sim_lru(const uint32_t* lines, int64_t n, int32_t sets, int32_t ways) {
    uint32_t* tag = malloc(sizeof(uint32_t) * (size_t)sets * ways);
    uint64_t* age = malloc(sizeof(uint64_t) * (size_t)sets * ways);
    for (int64_t i = 0; i < (int64_t)sets * ways; ++i) tag[i] = UINT32_MAX, age[i] = 0;
    int64_t miss = 0;
    for (int64_t i = 0; i < n; ++i) {
        const uint32_t l = lines[i];
        if (l == UINT32_MAX) continue;  /* no access */
        /* spread consecutive lines over the sets (the L2 hashes addresses over channels) */
        const uint32_t h = (l * 2654435761u) >> 7;
        const int64_t s = (int64_t)(h % (uint32_t)sets) * ways;
        int hit = -1, lru = 0;
        for (int w = 0; w < ways; ++w) {
            if (tag[s + w] == l) { hit = w; break; }
            if (age[s + w] < age[s + lru]) lru = w;
        }
        if (hit < 0) { ++miss; tag[s + lru] = l; hit = lru; }
        age[s + hit] = (uint64_t)i + 1;
    }
    free(tag);
    free(age);
    return miss;
}

// Host-side text helpers shared by the FASTA reader and the STS parser: strict
// UTF-8 decoding as Python's codec does it, and Python's str.isspace() set (the
// characters str.strip() removes).
#pragma once
#include <stdint.h>

namespace mp {

// Decode one UTF-8 code point at p (< end); returns its length or 0 if invalid
// (Python's strict decoder: no overlongs, no surrogates, <= U+10FFFF).
static inline int utf8_next(const uint8_t* p, const uint8_t* end, uint32_t* cp) {
    const uint8_t c = p[0];
    if (c < 0x80) { *cp = c; return 1; }
    if (c < 0xC2) return 0;
    if (c < 0xE0) {
        if (end - p < 2 || (p[1] & 0xC0) != 0x80) return 0;
        *cp = ((uint32_t)(c & 0x1F) << 6) | (p[1] & 0x3F);
        return 2;
    }
    if (c < 0xF0) {
        if (end - p < 3 || (p[1] & 0xC0) != 0x80 || (p[2] & 0xC0) != 0x80) return 0;
        if (c == 0xE0 && p[1] < 0xA0) return 0;   // overlong
        if (c == 0xED && p[1] >= 0xA0) return 0;  // surrogate
        *cp = ((uint32_t)(c & 0x0F) << 12) | ((uint32_t)(p[1] & 0x3F) << 6) | (p[2] & 0x3F);
        return 3;
    }
    if (c < 0xF5) {
        if (end - p < 4 || (p[1] & 0xC0) != 0x80 || (p[2] & 0xC0) != 0x80 || (p[3] & 0xC0) != 0x80) return 0;
        if (c == 0xF0 && p[1] < 0x90) return 0;   // overlong
        if (c == 0xF4 && p[1] >= 0x90) return 0;  // > U+10FFFF
        *cp = ((uint32_t)(c & 0x07) << 18) | ((uint32_t)(p[1] & 0x3F) << 12) | ((uint32_t)(p[2] & 0x3F) << 6) |
              (p[3] & 0x3F);
        return 4;
    }
    return 0;
}

static inline bool py_space(uint32_t cp) {
    if (cp < 0x80) return (cp >= 0x09 && cp <= 0x0D) || (cp >= 0x1C && cp <= 0x20);
    return cp == 0x85 || cp == 0xA0 || cp == 0x1680 || (cp >= 0x2000 && cp <= 0x200A) || cp == 0x2028 ||
           cp == 0x2029 || cp == 0x202F || cp == 0x205F || cp == 0x3000;
}

// Length of the code point ending just before `end` (>= begin), 0 if not a valid tail.
static inline int utf8_prev(const uint8_t* begin, const uint8_t* end, uint32_t* cp) {
    const uint8_t* p = end - 1;
    int n = 1;
    while (p > begin && n < 4 && (*p & 0xC0) == 0x80) { --p; ++n; }
    const int k = utf8_next(p, end, cp);
    return k == n ? k : 0;
}

}  // namespace mp

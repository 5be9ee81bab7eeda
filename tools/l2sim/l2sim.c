// l2sim.c -- trace-driven model of the y-form pass's per-XCD L2 behaviour
// (tools/l2sim/run.py drives it).  Each XCD has its own 4 MiB, 16-way,
// 128-B-line LRU L2; an XCD processes its own row list in order, and for
// every row touches: the row's CSR index lines (streamed), one 128-B line of
// the gathered table per nonzero, the own row of the table, the previous
// vector's row and the output row (write-allocate).  Reported: gather hit
// rate and the lines that miss L2 (what crosses to the fabric).
// Build: gcc -O2 -shared -fPIC l2sim.c -o libl2sim.so
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define WAYS 16

typedef struct {
    int64_t* tag;   // [sets][WAYS]
    uint32_t* age;  // LRU stamps
    int sets;
    uint32_t clock;
} Cache;

static int access_line(Cache* c, int64_t line) {
    const int s = (int)((uint64_t)line * 0x9E3779B97F4A7C15ULL >> 40) % c->sets;
    int64_t* t = c->tag + (int64_t)s * WAYS;
    uint32_t* a = c->age + (int64_t)s * WAYS;
    c->clock++;
    int victim = 0;
    for (int w = 0; w < WAYS; ++w) {
        if (t[w] == line) {
            a[w] = c->clock;
            return 1;
        }
        if (a[w] < a[victim]) victim = w;
    }
    t[victim] = line;
    a[victim] = c->clock;
    return 0;
}

// rowptr/col: CSR (int32 col), n rows.  order: concatenated per-XCD row
// lists, xcd_off[x]..xcd_off[x+1].  rowbytes: bytes of one table row (8P).
// Interleave: the XCD's rows are processed `inflight` at a time, one
// access of each in-flight row per turn (round robin), which models the
// waves' concurrent gathers.  out[0..5]: gathers, gather hits, stream
// lines, stream hits, csr lines, csr hits.
void simulate(int n, const int64_t* rowptr, const int32_t* col, const int32_t* order,
              const int64_t* xcd_off, int nxcd, int rowbytes, int l2_bytes, int inflight,
              int64_t* out, int stream_bypass) {
    memset(out, 0, sizeof(int64_t) * 6);
    const int64_t lines_per_row = (rowbytes + 127) / 128;
    const int64_t tbl = (int64_t)n * lines_per_row;  // line ids: table [0,tbl), yold [tbl,2tbl), out [2tbl,3tbl), csr above
    const int64_t csr_base = 3 * tbl;
    for (int x = 0; x < nxcd; ++x) {
        Cache c;
        c.sets = l2_bytes / 128 / WAYS;
        c.tag = (int64_t*)malloc(sizeof(int64_t) * c.sets * WAYS);
        c.age = (uint32_t*)calloc((size_t)c.sets * WAYS, sizeof(uint32_t));
        for (int64_t i = 0; i < (int64_t)c.sets * WAYS; ++i) c.tag[i] = -1;
        c.clock = 1;
        const int64_t b = xcd_off[x], e = xcd_off[x + 1];
        // window of in-flight rows: cursor per slot
        int64_t* slot_row = (int64_t*)malloc(sizeof(int64_t) * inflight);
        int64_t* slot_k = (int64_t*)malloc(sizeof(int64_t) * inflight);
        int64_t next = b;
        int active = 0;
        for (int s = 0; s < inflight; ++s) {
            if (next < e) {
                slot_row[s] = order[next++];
                slot_k[s] = -1;  // -1: row prologue (streams), then nonzeros
                active++;
            } else {
                slot_row[s] = -1;
            }
        }
        while (active > 0) {
            for (int s = 0; s < inflight; ++s) {
                const int64_t r = slot_row[s];
                if (r < 0) continue;
                if (slot_k[s] < 0) {  // own row, yold row, output row
                    for (int64_t l = 0; l < lines_per_row; ++l) {
                        out[2] += 3;
                        if (stream_bypass & 1) continue;  // streams do not allocate in L2
                        out[3] += access_line(&c, r * lines_per_row + l);
                        out[3] += access_line(&c, tbl + r * lines_per_row + l);
                        out[3] += access_line(&c, 2 * tbl + r * lines_per_row + l);
                    }
                    slot_k[s] = rowptr[r];
                }
                const int64_t k = slot_k[s];
                if (k < rowptr[r + 1]) {
                    out[4]++;
                    if (!(stream_bypass & 2)) out[5] += access_line(&c, csr_base + k / 32);
                    const int64_t cc = col[k];
                    for (int64_t l = 0; l < lines_per_row; ++l) {
                        out[0]++;
                        out[1] += access_line(&c, cc * lines_per_row + l);
                    }
                    slot_k[s] = k + 1;
                }
                if (slot_k[s] >= rowptr[r + 1]) {
                    if (next < e) {
                        slot_row[s] = order[next++];
                        slot_k[s] = -1;
                    } else {
                        slot_row[s] = -1;
                        active--;
                    }
                }
            }
        }
        free(slot_row);
        free(slot_k);
        free(c.tag);
        free(c.age);
    }
}

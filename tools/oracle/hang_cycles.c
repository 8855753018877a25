/* hang_cycles.c -- CPU experiment (test tooling; uses the oracle as the
 * checker only): do hang trials enter an exact architectural-state cycle?
 * If they did, a trial could be classified hang as soon as its state repeats
 * instead of running to the instruction cap.  Brent's cycle detection over
 * (pc, x[0..31], decoder state, stdout/stderr lengths, bytes stored: a cycle
 * only counts when nothing was stored inside it).
 *
 *   gcc -O2 -o /tmp/hang_cycles tools/oracle/hang_cycles.c -lpthread -lm
 *   /tmp/hang_cycles workloads/crc32.elf crc32 5000 0x5eed0002
 *
 * Result (round 1): crc32 seed 0x5eed0002, 5,000 trials -> 22 hangs, 0 exact
 * cycles.  The hangs are x31 (t6) flips of the table-builder loop counter:
 * the loop counts down from a huge value while t5 keeps changing, so no state
 * repeats.  Hang records also carry the pc at the cap (fi_outcome.detail), so
 * hang trials must be executed to the cap for bit-exact records.
 */
#include "../../oracle/rv64se.c"
#include <stdio.h>

typedef struct { u64 pc, x[32], fo, db, ol, el; int mid; u32 emi; int sap; } st_t;

static void snap(const mach_t *m, st_t *s) {
    s->pc = m->pc; memcpy(s->x, m->x, sizeof s->x); s->fo = m->fetch_offset; s->db = m->data_bytes;
    s->ol = m->out.len; s->el = m->err.len; s->mid = m->mid; s->emi = m->emi; s->sap = m->stay_at_pc;
}
static int same(const mach_t *m, const st_t *s) {
    return s->pc == m->pc && !memcmp(s->x, m->x, sizeof s->x) && s->fo == m->fetch_offset &&
           s->db == m->data_bytes && s->ol == m->out.len && s->el == m->err.len && s->mid == m->mid &&
           s->emi == m->emi && s->sap == m->stay_at_pc;
}

int main(int argc, char **argv) {
    if (argc < 5) { fprintf(stderr, "usage: %s elf argv0 n_trials seed\n", argv[0]); return 2; }
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 2; }
    static uint8_t buf[1 << 22];
    size_t n = fread(buf, 1, sizeof buf, f);
    fclose(f);
    or_campaign_t *c = or_create(buf, n, argv[2]);
    or_golden_t g;
    if (!c || or_golden(c, 1ULL << 32, &g)) { fprintf(stderr, "golden run failed\n"); return 1; }
    u64 N = strtoull(argv[3], 0, 0), seed = strtoull(argv[4], 0, 0);
    or_site_t *s = malloc(sizeof(or_site_t) * N);
    or_sample(c, seed, 0, N, 0x1fffffffeULL, 1, s);
    u64 cap = hang_cap(c, 0), sumdet = 0, sumcap = 0;
    int nh = 0, ncyc = 0;
    for (u64 i = 0; i < N; i++) {
        mach_t m; mach_init(&m, c); m.site = &s[i];
        st_t sv; int have = 0; u64 power = 1, lam = 0, det = 0;
        while (!m.done) {
            tick(&m, cap);
            if (!m.injected || m.done) continue;
            if (!have) { snap(&m, &sv); have = 1; continue; }
            lam++;
            if (!det && same(&m, &sv)) det = m.num_inst;
            if (lam == power) { snap(&m, &sv); power *= 2; lam = 0; }
        }
        if (m.res.cls == OR_HANG) {
            nh++; sumcap += cap - s[i].inst;
            if (det) { ncyc++; sumdet += det - s[i].inst; }
            else if (nh - ncyc <= 8)
                printf("no cycle: trial %u target %u inst %llu pc %llx\n", s[i].trial, s[i].target,
                       (unsigned long long)s[i].inst, (unsigned long long)m.pc);
        } else if (det) {
            printf("cycle but not hang: trial %llu cls %d\n", (unsigned long long)i, (int)m.res.cls);
        }
        mach_free(&m);
    }
    printf("hangs %d exact cycles %d (avg insts to detect %.0f, to cap %.0f)\n", nh, ncyc,
           ncyc ? (double)sumdet / ncyc : 0.0, nh ? (double)sumcap / nh : 0.0);
    return 0;
}

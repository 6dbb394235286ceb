// tools/sim/oca_sim.c -- SIMD schedule simulation of one wave's any_hit calls (the AO lambda of a user
// kernel: 64 lanes, one AO ray each, all entering any_hit together), on rays dumped by
// tools/sim/dump_ao_rays.py.  Counts wave-level vector loads (4 per pair-record visit, 3 per triangle
// test, the TD-bound unit of profiles/pmc_user_lambda.json) under:
//   P0  every lane walks its own ray (hip_kernels.h walk_slab: pop, descend to a leaf, test it)
//   P1  ordered cooperative walk: idle lanes take the bottom stack entry of lanes holding >= 2, every
//       entry carries its DFS-order key; a hit records (key, prim) per ray, work later in the ray's
//       order than its best hit is dropped; the answer is the smallest key = the reference's first hit
//   P1 with a descent cap (-c K): at most K node visits per iteration
// and checks that P1 returns every ray's P0 hit (hit / miss and the primitive).
//     gcc -O2 -o /tmp/oca_sim tools/sim/oca_sim.c -lm && /tmp/oca_sim /tmp/sim [cap]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float mn[3]; uint32_t first; float mx[3]; uint32_t n; } node_t;
typedef struct { uint32_t geom, prim, pad[2]; float v1[4], e1[4], e2[4]; } tri_t;
typedef struct { float o[3], d[3], inv[3], tmax; int valid; } ray_t;

static node_t* N; static tri_t* T;

static void* load(const char* dir, const char* f, size_t* n)
{
    char p[512]; snprintf(p, sizeof p, "%s/%s", dir, f);
    FILE* fp = fopen(p, "rb"); if (!fp) { perror(p); exit(1); }
    fseek(fp, 0, SEEK_END); *n = ftell(fp); fseek(fp, 0, SEEK_SET);
    void* m = malloc(*n); if (fread(m, 1, *n, fp) != *n) exit(2); fclose(fp); return m;
}

static int box(const node_t* b, const ray_t* r, float* tn)
{
    float t1x = (b->mn[0] - r->o[0]) * r->inv[0], t2x = (b->mx[0] - r->o[0]) * r->inv[0];
    float t1y = (b->mn[1] - r->o[1]) * r->inv[1], t2y = (b->mx[1] - r->o[1]) * r->inv[1];
    float t1z = (b->mn[2] - r->o[2]) * r->inv[2], t2z = (b->mx[2] - r->o[2]) * r->inv[2];
    float n = fmaxf(fmaxf(fminf(t1x, t2x), fminf(t1y, t2y)), fminf(t1z, t2z));
    float f = fminf(fminf(fmaxf(t1x, t2x), fmaxf(t1y, t2y)), fmaxf(t1z, t2z));
    *tn = n;
    return f >= n && f >= 0.0f && n < r->tmax;
}

static int tri(const tri_t* t, const ray_t* r)
{
    float e1[3] = { t->e1[0], t->e1[1], t->e1[2] }, e2[3] = { t->e2[0], t->e2[1], t->e2[2] };
    float s1[3] = { r->d[1] * e2[2] - r->d[2] * e2[1], r->d[2] * e2[0] - r->d[0] * e2[2], r->d[0] * e2[1] - r->d[1] * e2[0] };
    float div = s1[0] * e1[0] + s1[1] * e1[1] + s1[2] * e1[2];
    if (div == 0.0f) return 0;
    float inv = 1.0f / div;
    float d[3] = { r->o[0] - t->v1[0], r->o[1] - t->v1[1], r->o[2] - t->v1[2] };
    float b1 = (d[0] * s1[0] + d[1] * s1[1] + d[2] * s1[2]) * inv;
    if (b1 < 0.0f || b1 > 1.0f) return 0;
    float s2[3] = { d[1] * e1[2] - d[2] * e1[1], d[2] * e1[0] - d[0] * e1[2], d[0] * e1[1] - d[1] * e1[0] };
    float b2 = (r->d[0] * s2[0] + r->d[1] * s2[1] + r->d[2] * s2[2]) * inv;
    if (b2 < 0.0f || b1 + b2 > 1.0f) return 0;
    float tt = (e2[0] * s2[0] + e2[1] * s2[1] + e2[2] * s2[2]) * inv;
    return tt >= 0.0f && tt < r->tmax;
}

// one descent from `link` (node index; children at first, first + 1): visits counted, far children
// pushed (with the branch level), returns the leaf node reached or -1 (both children missed)
#define MAXS 64
typedef struct { uint32_t link[MAXS]; uint32_t lvl[MAXS]; int bot, top; } stack_t;

// DFS key: path bits MSB first, `len` bits, encoded with an end marker so that keys of disjoint
// subtrees compare lexicographically as integers
static uint64_t enc(uint64_t path, int len) { return (path << (40 - len)) | (1ull << (39 - len)); }

typedef struct {
    int task;              // ray (lane) worked on, -1 idle
    stack_t st;
    uint64_t path; int plen;
    uint32_t cur;          // node to resume (cap), or ~0u
} lane_t;

static long long vm0, vm1, it0, it1, calls, rays_total, don_total, mism, work_lane, sc0, sc1;
// per wave inner step: the node each descending lane visits (the scalar-fetch model: a step whose lanes
// all want the same pair record fetches it through the scalar cache, 0 vector loads)
static uint32_t seq[64][MAXS * 2];
static long long inner_cost(int* nv, int* act, long long* sc)
{
    int maxn = 0;
    for (int l = 0; l < 64; ++l) if (act[l] && nv[l] > maxn) maxn = nv[l];
    long long v = 0;
    for (int j = 0; j < maxn; ++j)
    {
        uint32_t first = ~0u; int uni = 1;
        for (int l = 0; l < 64; ++l)
        {
            if (!act[l] || nv[l] <= j) continue;
            if (first == ~0u) first = seq[l][j];
            else if (seq[l][j] != first) { uni = 0; break; }
        }
        if (uni) ++*sc; else v += 4;
    }
    return v;
}

// P0: independent lanes, walk_slab's SIMT shape; returns per ray the accepted prim (or ~0u)
static void p0(ray_t* R, uint32_t* ans)
{
    int st_top[64]; uint32_t stk[64][MAXS]; int done[64];
    for (int l = 0; l < 64; ++l) { done[l] = !R[l].valid; st_top[l] = 0; if (!done[l]) stk[l][st_top[l]++] = 0; ans[l] = ~0u; }
    for (;;)
    {
        int any = 0, maxn = 0, maxp = 0, NV[64] = {0}, ACT[64] = {0};
        for (int l = 0; l < 64; ++l)
        {
            if (done[l]) continue;
            if (st_top[l] == 0) { done[l] = 1; continue; }
            any = 1; ACT[l] = 1;
            uint32_t n = stk[l][--st_top[l]];
            int nv = 0, np = 0, leaf = 1;
            while (N[n].n == 0)
            {
                seq[l][nv] = n;
                ++nv; work_lane += 4;
                const node_t* c0 = &N[N[n].first]; const node_t* c1 = c0 + 1;
                float t0, t1; int b0 = box(c0, &R[l], &t0), b1 = box(c1, &R[l], &t1);
                if (!(b0 | b1)) { leaf = 0; break; }
                int go0 = (b0 & b1) ? (t0 < t1) : b0;
                if (b0 & b1) stk[l][st_top[l]++] = go0 ? N[n].first + 1 : N[n].first;
                n = go0 ? N[n].first : N[n].first + 1;
            }
            if (leaf)
                for (uint32_t i = N[n].first; i < N[n].first + N[n].n; ++i)
                {
                    ++np; work_lane += 3;
                    if (tri(&T[i], &R[l])) { ans[l] = i; done[l] = 1; break; }
                }
            NV[l] = nv;
            if (nv > maxn) maxn = nv;
            if (np > maxp) maxp = np;
        }
        if (!any) break;
        vm0 += inner_cost(NV, ACT, &sc0) + 3 * maxp; it0 += 1;
    }
}

// P1: ordered cooperative walk, descent cap `cap` (0 = none)
static void p1(ray_t* R, const uint32_t* ref, int cap)
{
    lane_t L[64]; uint64_t best[64]; uint32_t bprim[64];
    for (int l = 0; l < 64; ++l)
    {
        memset(&L[l], 0, sizeof L[l]);
        best[l] = ~0ull; bprim[l] = ~0u;
        L[l].task = R[l].valid ? l : -1; L[l].cur = ~0u;
        if (R[l].valid) { L[l].st.link[0] = 0; L[l].st.lvl[0] = 0; L[l].st.top = 1; }
    }
    for (;;)
    {
        // drop work later than its ray's best hit; segments with nothing left go idle
        for (int l = 0; l < 64; ++l)
        {
            lane_t* a = &L[l];
            if (a->task < 0) continue;
            if (a->cur == ~0u)
            {
                if (a->st.top == a->st.bot) { a->task = -1; continue; }
                const uint32_t lv = a->st.lvl[a->st.top - 1];
                const uint64_t kpath = ((a->path >> (a->plen - lv)) << 1) | 1ull;   // prefix(lv) + '1'
                if (lv > 0 || a->plen > 0) { if (enc(kpath, lv + 1) > best[a->task]) { a->task = -1; continue; } }
            }
            else if (enc(a->path, a->plen) > best[a->task]) { a->task = -1; continue; }
        }
        // donation: k-th idle lane <- bottom entry of the k-th lane with >= 2 entries
        int idle[64], ni = 0, donor[64], nd = 0;
        for (int l = 0; l < 64; ++l)
        {
            if (L[l].task < 0) idle[ni++] = l;
            else if (L[l].st.top - L[l].st.bot >= 2 || (getenv("DON1") && L[l].cur != ~0u && L[l].st.top - L[l].st.bot >= 1)) donor[nd++] = l;
        }
        const int nx = ni < nd ? ni : nd;
        for (int k = 0; k < nx; ++k)
        {
            lane_t* d = &L[donor[k]]; lane_t* h = &L[idle[k]];
            const uint32_t lk = d->st.link[d->st.bot], lv = d->st.lvl[d->st.bot];
            d->st.bot++;
            // the entry's key: the donor's path prefix of lv bits, then '1' (the far side)
            uint64_t pre = d->cur == ~0u && d->plen >= (int)lv ? d->path >> (d->plen - lv) : d->path >> (d->plen - lv);
            h->task = d->task; h->path = (pre << 1) | 1ull; h->plen = lv + 1;
            h->st.bot = 0; h->st.top = 0; h->cur = lk;
            ++don_total;
        }
        int any = 0, maxn = 0, maxp = 0, NV[64] = {0}, ACT[64] = {0};
        for (int l = 0; l < 64; ++l)
        {
            lane_t* a = &L[l];
            if (a->task < 0) continue;
            any = 1; ACT[l] = 1;
            ray_t* r = &R[a->task];
            uint32_t n;
            if (a->cur != ~0u) { n = a->cur; a->cur = ~0u; }
            else
            {
                const int k = --a->st.top;
                n = a->st.link[k];
                const uint32_t lv = a->st.lvl[k];
                a->path = ((a->path >> (a->plen - lv)) << 1) | 1ull;
                a->plen = lv + 1;
            }
            int nv = 0, np = 0, leaf = 1;
            while (N[n].n == 0)
            {
                if (cap && nv == cap) { a->cur = n; leaf = 0; break; }
                seq[l][nv] = n;
                ++nv;
                const node_t* c0 = &N[N[n].first]; const node_t* c1 = c0 + 1;
                float t0, t1; int b0 = box(c0, r, &t0), b1 = box(c1, r, &t1);
                if (!(b0 | b1)) { leaf = 0; break; }
                int go0 = (b0 & b1) ? (t0 < t1) : b0;
                if (b0 & b1)
                {
                    int k = a->st.top++;
                    a->st.link[k] = go0 ? N[n].first + 1 : N[n].first;
                    a->st.lvl[k] = a->plen;
                    a->path = a->path << 1;     // near side: '0'
                    a->plen += 1;
                }
                n = go0 ? N[n].first : N[n].first + 1;
            }
            if (leaf)
                for (uint32_t i = N[n].first; i < N[n].first + N[n].n; ++i)
                {
                    ++np;
                    if (tri(&T[i], r))
                    {
                        const uint64_t key = enc(a->path, a->plen);
                        if (key < best[a->task]) { best[a->task] = key; bprim[a->task] = i; }
                        a->task = -1;
                        break;
                    }
                }
            if (a->task >= 0 && a->cur == ~0u && a->st.top == a->st.bot) a->task = -1;
            NV[l] = nv;
            if (nv > maxn) maxn = nv;
            if (np > maxp) maxp = np;
        }
        if (!any) break;
        vm1 += inner_cost(NV, ACT, &sc1) + 3 * maxp; it1 += 1;
    }
    for (int l = 0; l < 64; ++l) if (R[l].valid && bprim[l] != ref[l]) ++mism;
}

int main(int argc, char** argv)
{
    const char* dir = argv[1];
    const int cap = argc > 2 ? atoi(argv[2]) : 0;
    size_t nb, tb, rb;
    N = load(dir, "nodes.bin", &nb); T = load(dir, "tris.bin", &tb);
    float* rr = load(dir, "rays.bin", &rb);
    const size_t groups = rb / (64 * 8 * 4);
    for (size_t g = 0; g < groups; ++g)
    {
        ray_t R[64]; uint32_t ans[64]; int nv = 0;
        for (int l = 0; l < 64; ++l)
        {
            const float* f = rr + (g * 64 + l) * 8;
            R[l].valid = f[0] != 0.0f;
            for (int k = 0; k < 3; ++k) { R[l].o[k] = f[1 + k]; R[l].d[k] = f[4 + k]; R[l].inv[k] = 1.0f / f[4 + k]; }
            R[l].tmax = f[7];
            nv += R[l].valid;
        }
        if (!nv) continue;
        ++calls; rays_total += nv;
        p0(R, ans);
        p1(R, ans, cap);
    }
    printf("calls %lld rays %lld | P0 vmem %.1f/call iters %.1f | P1(cap %d) vmem %.1f/call iters %.1f donations %.1f/call | "
           "vmem ratio %.3f | mismatches %lld | ideal %.1f/call | scalar steps P0 %.1f P1 %.1f\n", calls, rays_total, (double)vm0 / calls, (double)it0 / calls, cap,
           (double)vm1 / calls, (double)it1 / calls, (double)don_total / calls, (double)vm1 / vm0, mism,
           (double)work_lane / 64.0 / calls, (double)sc0 / calls, (double)sc1 / calls);
    return 0;
}

/* ASan/UBSan driver for the CPU oracle and the optimised CPU baseline
 * (oracle/ewal_oracle.c, oracle/ewal_cpu_fast.c): random WALs through the
 * writer, every single-byte corruption class through ReadAll, random bytes
 * through every Unmarshal / proto.Skip, snapshots and maybeCommit.  Built and
 * run by tests/test_sanitizers.py (the reference runs its tests
 * under `go test --race`). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/ewal_cpu_fast.h"
#include "../../oracle/ewal_oracle.h"

static uint64_t rs = 88172645463325252ull;
static uint64_t rnd(void) {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}

static uint8_t *build_wal(int n, int maxd, int64_t *len) {
  or_encoder e;
  or_encoder_init(&e, 0);
  or_encode(&e, 4, NULL, 0, 1);
  or_encode(&e, 1, (const uint8_t *)"md", 2, 0);
  uint8_t st[64];
  int64_t sl = or_hardstate_marshal(1, 2, 3, st);
  or_encode(&e, 3, st, sl, 0);
  uint8_t *d = malloc((size_t)maxd + 64), *ent = malloc((size_t)maxd + 128);
  for (int i = 0; i < n; i++) {
    int dl = (int)(rnd() % (uint64_t)(maxd + 1));
    for (int k = 0; k < dl; k++) d[k] = (uint8_t)rnd();
    int64_t el = or_entry_marshal(0, 1, (uint64_t)i + 1, dl ? d : NULL, dl, ent);
    or_encode(&e, 2, ent, el, 0);
  }
  free(d);
  free(ent);
  *len = e.len;
  uint8_t *out = malloc((size_t)e.len + 1);
  memcpy(out, e.buf, (size_t)e.len);
  or_encoder_free(&e);
  return out;
}

int main(void) {
  int checks = 0;
  for (int t = 0; t < 40; t++) {
    int64_t n;
    uint8_t *w = build_wal((int)(rnd() % 40), (int)(rnd() % 2000), &n);
    for (int m = 0; m < 60; m++) {
      uint8_t *c = malloc((size_t)n + 1);
      memcpy(c, w, (size_t)n);
      int64_t cut = n;
      if (n && m % 3 == 0) c[rnd() % (uint64_t)n] ^= (uint8_t)(1u << (rnd() % 8));
      if (n && m % 3 == 1) c[rnd() % (uint64_t)n] = (uint8_t)rnd();
      if (n && m % 5 == 2) cut = (int64_t)(rnd() % (uint64_t)n);
      or_readall_result r;
      or_readall(c, cut, rnd() % 3, &r);
      or_readall_free(&r);
      orf_result f;
      orf_readall(c, cut, 1, 2, &f);
      orf_result_free(&f);
      uint32_t crcs[64];
      int64_t offs[64];
      or_chain_crcs(c, cut, crcs, 64, offs);
      free(c);
      checks++;
    }
    free(w);
  }
  /* random bytes through every Unmarshal and proto.Skip */
  uint8_t buf[512];
  for (int t = 0; t < 20000; t++) {
    int64_t l = (int64_t)(rnd() % 64);
    for (int k = 0; k < l; k++) buf[k] = (uint8_t)(rnd() % 4 == 0 ? rnd() % 0x30 : rnd());
    or_record r; memset(&r, 0, sizeof(r)); or_record_unmarshal(buf, l, &r); or_record_free(&r);
    or_entry e; memset(&e, 0, sizeof(e)); or_entry_unmarshal(buf, l, &e); or_entry_free(&e);
    or_hardstate h; memset(&h, 0, sizeof(h)); or_hardstate_unmarshal(buf, l, &h); or_hardstate_free(&h);
    or_snapshot s; memset(&s, 0, sizeof(s)); or_snapshot_unmarshal(buf, l, &s); or_snapshot_free(&s);
    or_snappb p; memset(&p, 0, sizeof(p)); or_snappb_unmarshal(buf, l, &p); or_snappb_free(&p);
    or_message g; memset(&g, 0, sizeof(g)); or_message_unmarshal(buf, l, &g); or_message_free(&g);
    int64_t sk; or_proto_skip(buf, l, &sk);
    or_loadsnap_result ls; or_loadsnap(buf, l, OR_CASTAGNOLI, &ls); or_loadsnap_free(&ls);
    checks++;
  }
  /* CRC paths agree */
  for (int t = 0; t < 200; t++) {
    size_t l = (size_t)(rnd() % 40000);
    uint8_t *d = malloc(l + 1);
    for (size_t k = 0; k < l; k++) d[k] = (uint8_t)rnd();
    uint32_t s = (uint32_t)rnd();
    if (or_crc32_update(s, OR_CASTAGNOLI, d, l) != or_crc32_update_table(s, OR_CASTAGNOLI, d, l) ||
        orf_crc32c_update(s, d, l) != or_crc32_update(s, OR_CASTAGNOLI, d, l)) {
      fprintf(stderr, "crc mismatch\n");
      return 1;
    }
    free(d);
  }
  /* maybeCommit, single and batched */
  uint64_t G = 500, match[9 * 500], term[500], com[500], com2[500], off[500], ptr[501], lt[500 * 8];
  uint8_t nv[500], ch[500], st[500], ch2[500], st2[500];
  for (uint64_t g = 0; g < G; g++) {
    nv[g] = (uint8_t)(rnd() % 10);
    for (int v = 0; v < 9; v++) match[v * G + g] = rnd() % 30;
    term[g] = 1 + rnd() % 3;
    com[g] = com2[g] = rnd() % 20;
    off[g] = rnd() % 5;
    ptr[g] = g * 8;
    for (int k = 0; k < 8; k++) lt[g * 8 + k] = 1 + rnd() % 3;
  }
  ptr[G] = G * 8;
  or_maybe_commit_batch(G, match, nv, term, com, off, ptr, lt, ch, st);
  orf_maybe_commit_batch(G, match, nv, term, com2, off, ptr, lt, ch2, st2, 3);
  if (memcmp(com, com2, sizeof(com)) || memcmp(ch, ch2, sizeof(ch)) || memcmp(st, st2, sizeof(st))) {
    fprintf(stderr, "commit mismatch\n");
    return 1;
  }
  printf("san_oracle ok: %d cases\n", checks);
  return 0;
}

// ingress_host.cpp — host-side ingress helper for the aggregator (no GPU code): strip the large byte
// strings out of an executor's pickled result so that it can be unpickled without copying them.
//
// The executor ships every client update as pickle.dumps(results) (torch_client.py:79-91, protocol 4),
// and the reference aggregator unpickles it on its event-loop thread (aggregator.py:704,994):
// pickle.loads copies each numpy array's raw bytes out of the payload, single-threaded — 45 MB per
// ResNet-18 update, most of the aggregator's per-update host time.  fa_pickle_strip walks
// the opcode stream (every opcode of protocols 0-4 has a self-describing argument length), drops the
// optional FRAME opcodes, and replaces each BINBYTES / BINBYTES8 / BYTEARRAY8 argument of at least
// `min_bytes` by a 12-byte SHORT_BINBYTES tag ("FAPB" + region index).  The stripped stream (a few KiB)
// is unpickled normally; fedscale_amd/ingress.py turns the tagged arrays into zero-copy views of the
// payload, which the native gather then copies straight into pinned staging, multi-threaded.
#include <stdint.h>
#include <string.h>

#include "../../include/fedagg.h"

extern "C" __attribute__((visibility("hidden"))) int fa_internal_set_error(int code, const char* msg);

namespace {

enum ArgKind : uint8_t {
  A_NONE,
  A_FIX1, A_FIX2, A_FIX4, A_FIX8,   // fixed-size argument
  A_LEN1, A_LEN4, A_LEN8,           // length-prefixed (1 / 4 / 8-byte little-endian length)
  A_BYTES4, A_BYTES8,               // length-prefixed byte strings we may strip
  A_NL1, A_NL2,                     // one / two newline-terminated lines
  A_BAD,                            // unknown, or out-of-band buffers (protocol 5): not handled
};

struct Table {
  ArgKind k[256];
  Table() {
    for (int i = 0; i < 256; ++i) k[i] = A_BAD;
    const char* none = "N\x88\x89]ael)t\x85\x86\x87}dsu\x8f\x90\x91" "0" "2(1\x94\x93Rbo\x81\x92.Q";
    for (const char* p = none; *p; ++p) k[(uint8_t)*p] = A_NONE;
    k[(uint8_t)'K'] = A_FIX1; k[(uint8_t)'h'] = A_FIX1; k[(uint8_t)'q'] = A_FIX1; k[0x82] = A_FIX1;
    k[0x80] = A_FIX1;                                       // PROTO
    k[(uint8_t)'M'] = A_FIX2; k[0x83] = A_FIX2;
    k[(uint8_t)'J'] = A_FIX4; k[(uint8_t)'j'] = A_FIX4; k[(uint8_t)'r'] = A_FIX4; k[0x84] = A_FIX4;
    k[(uint8_t)'G'] = A_FIX8; k[0x95] = A_FIX8;             // BINFLOAT, FRAME
    k[0x8a] = A_LEN1; k[(uint8_t)'U'] = A_LEN1; k[(uint8_t)'C'] = A_LEN1; k[0x8c] = A_LEN1;
    k[0x8b] = A_LEN4; k[(uint8_t)'T'] = A_LEN4; k[(uint8_t)'X'] = A_LEN4;
    k[0x8d] = A_LEN8;
    k[(uint8_t)'B'] = A_BYTES4;
    k[0x8e] = A_BYTES8; k[0x96] = A_BYTES8;
    const char* nl1 = "ILSVFgpP";
    for (const char* p = nl1; *p; ++p) k[(uint8_t)*p] = A_NL1;
    k[(uint8_t)'c'] = A_NL2; k[(uint8_t)'i'] = A_NL2;
  }
};
const Table kTable;

uint64_t rd_le(const uint8_t* p, int nb) {
  uint64_t v = 0;
  for (int i = nb - 1; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

int fail(int code, const char* msg) { return fa_internal_set_error(code, msg); }

}  // namespace

extern "C" int64_t fa_pickle_strip(const uint8_t* in, int64_t n, int64_t min_bytes, uint8_t* out, int64_t out_cap,
                                   int64_t* regions, int32_t max_regions, int32_t* nregions) {
  if (!in || n < 0 || !nregions || max_regions < 0 || (max_regions > 0 && !regions) || min_bytes < 16)
    return fail(FA_E_ARG, "fa_pickle_strip: bad arguments");
  int64_t i = 0, o = 0;
  int32_t nr = 0;
  bool stopped = false;
  auto emit = [&](const uint8_t* p, int64_t len) {
    if (out && o + len <= out_cap) memcpy(out + o, p, (size_t)len);
    o += len;
  };
  while (i < n) {
    const uint8_t op = in[i];
    const ArgKind kind = kTable.k[op];
    int64_t arg = 0;  // bytes after the opcode
    switch (kind) {
      case A_BAD: return fail(FA_E_RANGE, "fa_pickle_strip: unsupported opcode");
      case A_NONE: arg = 0; break;
      case A_FIX1: arg = 1; break;
      case A_FIX2: arg = 2; break;
      case A_FIX4: arg = 4; break;
      case A_FIX8: arg = 8; break;
      case A_LEN1:
        if (i + 2 > n) return fail(FA_E_RANGE, "fa_pickle_strip: truncated");
        arg = 1 + (int64_t)in[i + 1];
        break;
      case A_LEN4:
      case A_BYTES4:
        if (i + 5 > n) return fail(FA_E_RANGE, "fa_pickle_strip: truncated");
        arg = 4 + (int64_t)(uint32_t)rd_le(in + i + 1, 4);
        break;
      case A_LEN8:
      case A_BYTES8: {
        if (i + 9 > n) return fail(FA_E_RANGE, "fa_pickle_strip: truncated");
        const uint64_t len = rd_le(in + i + 1, 8);
        if (len > (uint64_t)n) return fail(FA_E_RANGE, "fa_pickle_strip: bad length");
        arg = 8 + (int64_t)len;
        break;
      }
      case A_NL1:
      case A_NL2: {
        int lines = kind == A_NL1 ? 1 : 2;
        int64_t j = i + 1;
        while (lines > 0 && j < n) {
          if (in[j] == '\n') --lines;
          ++j;
        }
        if (lines > 0) return fail(FA_E_RANGE, "fa_pickle_strip: truncated line");
        arg = j - i - 1;
        break;
      }
    }
    if (i + 1 + arg > n) return fail(FA_E_RANGE, "fa_pickle_strip: truncated argument");
    if (op == 0x95) {  // FRAME: an optional framing hint; dropped (the unpickler accepts unframed streams)
      i += 1 + arg;
      continue;
    }
    const int hdr = kind == A_BYTES4 ? 4 : 8;
    if ((kind == A_BYTES4 || kind == A_BYTES8) && arg - hdr >= min_bytes && op != 0x96) {
      if (nr < max_regions) {
        regions[2 * nr] = i + 1 + hdr;  // offset of the raw bytes in `in`
        regions[2 * nr + 1] = arg - hdr;
      }
      uint8_t tag[14] = {'C', 12, 'F', 'A', 'P', 'B'};
      const uint64_t idx = (uint64_t)nr;
      for (int b = 0; b < 8; ++b) tag[6 + b] = (uint8_t)(idx >> (8 * b));
      emit(tag, 14);
      ++nr;
    } else {
      emit(in + i, 1 + arg);
    }
    i += 1 + arg;
    if (op == '.') {
      stopped = true;
      break;
    }
  }
  if (!stopped) return fail(FA_E_RANGE, "fa_pickle_strip: no STOP opcode");
  *nregions = nr;
  return o;  // bytes of the stripped stream (it was written only if it fit in out_cap)
}

/**
 * A gzip writer whose output is a function of its input alone.
 *
 * The plugin archive's sha256 is committed to artifacthub-pkg.yml and
 * re-derived by the CPU gate and by the release job. zlib's deflate output is
 * not stable across builds of zlib (Node 12 bundles zlib 1.2.11, Node 20 a
 * Chromium fork with different match finding), so the same tree would hash
 * differently on this container and on the release runner. This encoder is
 * plain JavaScript: greedy LZ77 over a 32 KiB window with 3-byte hash chains,
 * one final block of fixed Huffman codes (RFC 1951 §3.2.6), in a gzip member
 * with mtime 0 (RFC 1952). Any inflater reads it; the bytes depend on nothing
 * but the input.
 */

const WINDOW = 32768;
const MIN_MATCH = 3;
const MAX_MATCH = 258;
const MAX_CHAIN = 128;
const HASH_BITS = 15;
const HASH_SIZE = 1 << HASH_BITS;

// RFC 1951 §3.2.5: length codes 257..285 and distance codes 0..29.
const LEN_BASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258];
const LEN_EXTRA = [0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0];
const DIST_BASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
  6145, 8193, 12289, 16385, 24577];
const DIST_EXTRA = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13];

// length 3..258 → code index; distance 1..32768 → code index
const LEN_CODE = new Uint8Array(MAX_MATCH + 1);
for (let c = 0; c < LEN_BASE.length; c++) {
  const hi = c + 1 < LEN_BASE.length ? LEN_BASE[c + 1] : MAX_MATCH + 1;
  for (let l = LEN_BASE[c]; l < hi && l <= MAX_MATCH; l++) LEN_CODE[l] = c;
}
LEN_CODE[MAX_MATCH] = LEN_BASE.length - 1;
function distCode(d) {
  let lo = 0;
  let hi = DIST_BASE.length - 1;
  while (lo < hi) {
    const mid = (lo + hi + 1) >> 1;
    if (DIST_BASE[mid] <= d) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

/** Fixed literal/length code of symbol s → [reversed code, bit length] (Huffman codes go MSB first). */
function reverse(code, len) {
  let r = 0;
  for (let i = 0; i < len; i++) {
    r = (r << 1) | (code & 1);
    code >>>= 1;
  }
  return r;
}
const LIT_CODE = new Uint16Array(288);
const LIT_LEN = new Uint8Array(288);
for (let s = 0; s < 288; s++) {
  let code;
  let len;
  if (s < 144) { code = 0x30 + s; len = 8; }
  else if (s < 256) { code = 0x190 + (s - 144); len = 9; }
  else if (s < 280) { code = s - 256; len = 7; }
  else { code = 0xc0 + (s - 280); len = 8; }
  LIT_CODE[s] = reverse(code, len);
  LIT_LEN[s] = len;
}
const DIST_REV = new Uint8Array(30);
for (let d = 0; d < 30; d++) DIST_REV[d] = reverse(d, 5);

function BitWriter(cap) {
  this.buf = new Uint8Array(cap);
  this.pos = 0;
  this.bits = 0;
  this.n = 0;
}
BitWriter.prototype.put = function (value, len) {
  this.bits |= value << this.n;
  this.n += len;
  while (this.n >= 8) {
    if (this.pos === this.buf.length) {
      const next = new Uint8Array(this.buf.length * 2);
      next.set(this.buf);
      this.buf = next;
    }
    this.buf[this.pos++] = this.bits & 0xff;
    this.bits >>>= 8;
    this.n -= 8;
  }
};
BitWriter.prototype.finish = function () {
  if (this.n > 0) this.put(0, 8 - this.n);
  return this.buf.subarray(0, this.pos);
};

/** Raw deflate stream (one final fixed-Huffman block) of `data` (Uint8Array). */
export function deflateRaw(data) {
  const n = data.length;
  const w = new BitWriter(Math.max(1024, n >> 1));
  w.put(1, 1); // BFINAL
  w.put(1, 2); // BTYPE 01: fixed Huffman
  const head = new Int32Array(HASH_SIZE).fill(-1);
  const prev = new Int32Array(WINDOW);
  function hash(i) {
    return ((data[i] << 10) ^ (data[i + 1] << 5) ^ data[i + 2]) & (HASH_SIZE - 1);
  }
  function insert(i) {
    if (i + MIN_MATCH > n) return;
    const h = hash(i);
    prev[i & (WINDOW - 1)] = head[h];
    head[h] = i;
  }
  function literal(b) { w.put(LIT_CODE[b], LIT_LEN[b]); }
  let i = 0;
  while (i < n) {
    let bestLen = 0;
    let bestDist = 0;
    if (i + MIN_MATCH <= n) {
      const limit = Math.min(MAX_MATCH, n - i);
      let cand = head[hash(i)];
      let chain = MAX_CHAIN;
      while (cand >= 0 && i - cand <= WINDOW && chain-- > 0) {
        if (data[cand + bestLen] === data[i + bestLen]) {
          let l = 0;
          while (l < limit && data[cand + l] === data[i + l]) l++;
          if (l > bestLen) {
            bestLen = l;
            bestDist = i - cand;
            if (l === limit) break;
          }
        }
        const p = prev[cand & (WINDOW - 1)];
        if (p >= cand) break; // the slot was overwritten by a newer position: the chain left the window
        cand = p;
      }
    }
    if (bestLen >= MIN_MATCH) {
      const lc = LEN_CODE[bestLen];
      w.put(LIT_CODE[257 + lc], LIT_LEN[257 + lc]);
      if (LEN_EXTRA[lc]) w.put(bestLen - LEN_BASE[lc], LEN_EXTRA[lc]);
      const dc = distCode(bestDist);
      w.put(DIST_REV[dc], 5);
      if (DIST_EXTRA[dc]) w.put(bestDist - DIST_BASE[dc], DIST_EXTRA[dc]);
      for (let k = 0; k < bestLen; k++) insert(i + k);
      i += bestLen;
    } else {
      literal(data[i]);
      insert(i);
      i++;
    }
  }
  w.put(LIT_CODE[256], LIT_LEN[256]); // end of block
  return w.finish();
}

const CRC_TABLE = new Int32Array(256);
for (let k = 0; k < 256; k++) {
  let c = k;
  for (let j = 0; j < 8; j++) c = c & 1 ? 0xedb88320 ^ (c >>> 1) : c >>> 1;
  CRC_TABLE[k] = c;
}

export function crc32(data) {
  let c = -1;
  for (let i = 0; i < data.length; i++) c = CRC_TABLE[(c ^ data[i]) & 0xff] ^ (c >>> 8);
  return (c ^ -1) >>> 0;
}

/** A single-member gzip file of `data` (Buffer / Uint8Array) → Buffer. mtime 0, OS 3 (Unix), no name. */
export function gzipStable(data) {
  const body = deflateRaw(data);
  const out = Buffer.alloc(10 + body.length + 8);
  out[0] = 0x1f;
  out[1] = 0x8b;
  out[2] = 8; // CM deflate
  out[3] = 0; // FLG
  out.writeUInt32LE(0, 4); // MTIME
  out[8] = 0; // XFL
  out[9] = 3; // OS
  Buffer.from(body.buffer, body.byteOffset, body.length).copy(out, 10);
  out.writeUInt32LE(crc32(data), 10 + body.length);
  out.writeUInt32LE(data.length >>> 0, 14 + body.length);
  return out;
}

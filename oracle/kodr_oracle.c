/*
 * kodr_oracle.c -- CPU restatement of itzmeanjan/kodr's RLNC arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP engine
 * in kodr_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product library (libkodr_rlnc.so) never
 * links, loads or calls anything in oracle/.
 *
 * It restates kodr's Go code path line by line as scalar C (same per-byte zero
 * checks and LOG/EXP table lookups), so it is also the "kodr-equivalent scalar
 * path" timed as the CPU baseline (kodr itself is Go and there is no Go
 * toolchain in this image or on the GPU box).  Citations are
 * path:line relative to the reference checkout.
 *
 * Pinning: the field tables are the literal tables of
 * kodr_internals/gf256/gf256.go:15-44 (tests/golden/gf256_tables.json, parsed
 * from that file's text and also regenerated from x^8+x^4+x^3+x^2+1 here);
 * matrix multiply / RREF / rank results are checked against the known-answer
 * tests of kodr_internals/matrix/matrix_test.go:12-109 and IsSystematic against
 * kodr_internals/data_test.go:136-156 (tests/test_oracle.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* error codes == position in errors.go:6-17 (1-based) */
enum {
    OK = 0,
    ERR_CANNOT_INVERT = 1,          /* errors.go:6  */
    ERR_MATRIX_DIM = 2,             /* errors.go:7  */
    ERR_ALL_USEFUL_RECEIVED = 3,    /* errors.go:8  */
    ERR_MORE_USEFUL_REQUIRED = 4,   /* errors.go:9  */
    ERR_COPY_FAILED = 5,            /* errors.go:10 */
    ERR_PIECE_COUNT_GT_BYTES = 6,   /* errors.go:11 */
    ERR_ZERO_PIECE_SIZE = 7,        /* errors.go:12 */
    ERR_BAD_PIECE_COUNT = 8,        /* errors.go:13 */
    ERR_CODED_LEN_MISMATCH = 9,     /* errors.go:14 */
    ERR_VECTOR_LEN_MISMATCH = 10,   /* errors.go:15 */
    ERR_NOT_DECODED_YET = 11,       /* errors.go:16 */
    ERR_PIECE_OUT_OF_BOUND = 12,    /* errors.go:17 */
};

/* ---------------------------------------------------------------- field -- */
/* gf256.go:15-44: LOG[256], EXP[510] for poly 0x11D, generator 2. */
static uint8_t LOG[256];
static uint8_t EXP[510];
static int tables_ready = 0;

static void build_tables(void) {
    if (tables_ready) return;
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        EXP[i] = (uint8_t)x;
        LOG[x] = (uint8_t)i;
        x <<= 1;
        if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 510; i++) EXP[i] = EXP[i - 255];
    LOG[0] = 0; /* gf256.go:16 first entry; never used (Mul short-circuits zero) */
    tables_ready = 1;
}

void oracle_tables(uint8_t log_out[256], uint8_t exp_out[510]) {
    build_tables();
    memcpy(log_out, LOG, 256);
    memcpy(exp_out, EXP, 510);
}

/* gf256.go:109-118 */
static inline uint8_t gf_mul(uint8_t a, uint8_t b) {
    if (a == 0 || b == 0) return 0;
    return EXP[(int)LOG[a] + (int)LOG[b]];
}

uint8_t oracle_gf_mul(uint8_t a, uint8_t b) { build_tables(); return gf_mul(a, b); }

/* gf256.go:77-86 */
int oracle_gf_inv(uint8_t a, uint8_t* out) {
    build_tables();
    if (a == 0) return ERR_CANNOT_INVERT;
    *out = EXP[255 - LOG[a]];
    return OK;
}

/* gf256.go:121-127 */
int oracle_gf_div(uint8_t a, uint8_t b, uint8_t* out) {
    uint8_t inv;
    if (oracle_gf_inv(b, &inv) != OK) return ERR_CANNOT_INVERT;
    *out = gf_mul(a, inv);
    return OK;
}

/* ------------------------------------------------------------ data.go -- */
/* data.go:19-29  Piece.Multiply: p[i] ^= src[i] * by */
void oracle_piece_multiply(uint8_t* dst, const uint8_t* src, size_t n, uint8_t by) {
    build_tables();
    for (size_t i = 0; i < n; i++) dst[i] ^= gf_mul(src[i], by);
}

/* data.go:137-166  OriginalPiecesFromDataAndPieceCount -> (pieceSize, padding) */
int oracle_split_by_count(size_t len, size_t piece_count, size_t* piece_size, size_t* padding) {
    if (piece_count < 2) return ERR_BAD_PIECE_COUNT;                  /* :138-140 */
    if (piece_count > len) return ERR_PIECE_COUNT_GT_BYTES;           /* :142-144 */
    size_t ps = (len + (piece_count - 1)) / piece_count;              /* :146 */
    size_t pad = piece_count * ps - len;                              /* :147 */
    /* :164 re-splits the padded buffer by size; that call can only fail when
     * ps >= padded length, i.e. a single piece, excluded by piece_count>=2 */
    if (ps >= ps * piece_count) return ERR_BAD_PIECE_COUNT;
    *piece_size = ps;
    *padding = pad;
    return OK;
}

/* data.go:103-132  OriginalPiecesFromDataAndPieceSize -> (pieceCount, padding) */
int oracle_split_by_size(size_t len, size_t piece_size, size_t* piece_count, size_t* padding) {
    if (piece_size == 0) return ERR_ZERO_PIECE_SIZE;                  /* :104-106 */
    if (piece_size >= len) return ERR_BAD_PIECE_COUNT;                /* :108-110 */
    size_t pc = (len + piece_size - 1) / piece_size;                  /* :112 math.Ceil */
    *piece_count = pc;
    *padding = pc * piece_size - len;                                 /* :113 */
    return OK;
}

/* data.go:64-84  CodedPiece.IsSystematic */
int oracle_is_systematic(const uint8_t* vec, size_t n) {
    long pos = -1;
    for (size_t i = 0; i < n; i++) {
        if (vec[i] == 0) continue;
        if (vec[i] == 1) {
            if (pos != -1) return 0;
            pos = (long)i;
        } else {
            return 0;
        }
    }
    return pos >= 0 && (size_t)pos < n;
}

/* data.go:173-193  CodedPiecesForRecoding: validation only (slicing is views) */
int oracle_coded_pieces_for_recoding(size_t data_len, size_t piece_count, size_t coded_together,
                                     size_t* coded_piece_len) {
    if (piece_count == 0) return ERR_CODED_LEN_MISMATCH; /* Go would divide by zero and panic */
    size_t cpl = data_len / piece_count;                              /* :174 */
    if (cpl * piece_count != data_len) return ERR_CODED_LEN_MISMATCH; /* :175-177 */
    if (!(coded_together < cpl)) return ERR_VECTOR_LEN_MISMATCH;      /* :179-181 */
    *coded_piece_len = cpl;
    return OK;
}

/* ----------------------------------------------------------- encoders -- */
/* full/encoder.go:61-71: out = sum_i v[i] * P_i, one coded piece per vector.
 * pieces: k rows of L bytes, contiguous (data.go:121-128 slices one buffer). */
void oracle_encode(const uint8_t* pieces, size_t k, size_t L,
                   const uint8_t* vecs, size_t B, uint8_t* out) {
    build_tables();
    for (size_t b = 0; b < B; b++) {
        uint8_t* piece = out + b * L;
        memset(piece, 0, L);                                          /* :63 make() */
        for (size_t i = 0; i < k; i++)                                /* :64-66 */
            oracle_piece_multiply(piece, pieces + i * L, L, vecs[b * k + i]);
    }
}

/* matrix.go:45-69  Matrix.Multiply (m: ar x ac, with: br x bc) */
int oracle_matmul(const uint8_t* m, size_t ar, size_t ac,
                  const uint8_t* w, size_t br, size_t bc, uint8_t* out) {
    build_tables();
    if (ac != br) return ERR_MATRIX_DIM;                              /* :46-48 */
    memset(out, 0, ar * bc);
    for (size_t i = 0; i < ar; i++)
        for (size_t j = 0; j < bc; j++)
            for (size_t k = 0; k < ac; k++)
                out[i * bc + j] ^= gf_mul(m[i * ac + k], w[k * bc + j]);
    return OK;
}

/* full/recoder.go:27-46 over a flattened buffer (recoder.go:63-70 +
 * data.go:173-193).  flat: n coded pieces of clen = k + L bytes, wire layout
 * vector ++ piece.  r: B recoding vectors of n bytes.  out: B x clen. */
int oracle_recode(const uint8_t* flat, size_t n, size_t k, size_t clen,
                  const uint8_t* r, size_t B, uint8_t* out) {
    build_tables();
    if (k >= clen) return ERR_VECTOR_LEN_MISMATCH;
    size_t L = clen - k;
    size_t csz = n * k;
    uint8_t* C = (uint8_t*)malloc(csz > 0 ? csz : 1);                  /* fill() :13-22 */
    for (size_t i = 0; i < n; i++) memcpy(C + i * k, flat + i * clen, k);
    for (size_t b = 0; b < B; b++) {
        uint8_t* vec = out + b * clen;
        uint8_t* piece = vec + k;
        memset(piece, 0, L);                                          /* :30 */
        for (size_t i = 0; i < n; i++)                                /* :32-34 */
            oracle_piece_multiply(piece, flat + i * clen + k, L, r[b * n + i]);
        oracle_matmul(r + b * n, 1, n, C, n, k, vec);                 /* :36-40 */
    }
    free(C);
    return OK;
}

/* systematic/encoder.go:82-109 for a run of B calls starting at call index
 * `start_id`: calls < k emit (e_id, copy P_id) (:83-96), later calls consume the
 * next caller-supplied random vector (:98-108).  vecs holds one k-byte vector
 * per output; entries for systematic outputs are overwritten with e_id. */
void oracle_systematic_encode(const uint8_t* pieces, size_t k, size_t L, size_t start_id,
                              uint8_t* vecs, size_t B, uint8_t* out) {
    build_tables();
    for (size_t b = 0; b < B; b++) {
        size_t id = start_id + b;
        if (id < k) {
            memset(vecs + b * k, 0, k);                               /* :60-68 */
            vecs[b * k + id] = 1;
            memcpy(out + b * L, pieces + id * L, L);                  /* :88-89 */
        } else {
            oracle_encode(pieces, k, L, vecs + b * k, 1, out + b * L);
        }
    }
}

/* ------------------------------------------------------ decoder state -- */
/* kodr_internals/matrix/decoder_state.go:9-13.  Rows are separately owned
 * buffers addressed through pointer arrays so that swaps and removals move
 * pointers exactly like the Go slice-of-slices does. */
typedef struct {
    size_t piece_count;      /* :10 */
    size_t rows, cap;
    size_t cols;             /* coefficient columns (len of first vector) */
    size_t plen;             /* coded piece length */
    uint8_t** coeffs;        /* :11 */
    uint8_t** coded;         /* :12 */
    /* full/decoder.go:11-14 */
    size_t expected, useful, received;
} oracle_decoder;

static void ds_clean_forward(oracle_decoder* d) {                      /* :15-76 */
    long rows = (long)d->rows, cols = (long)d->cols;
    long boundary = rows < cols ? rows : cols;
    for (long i = 0; i < boundary; i++) {
        if (d->coeffs[i][i] == 0) {
            int non_zero_col = 0;
            long pivot = i + 1;
            for (; pivot < rows; pivot++) {
                if (d->coeffs[pivot][i] != 0) { non_zero_col = 1; break; }
            }
            if (!non_zero_col) continue;
            uint8_t* t = d->coeffs[i]; d->coeffs[i] = d->coeffs[pivot]; d->coeffs[pivot] = t;
            t = d->coded[i]; d->coded[i] = d->coded[pivot]; d->coded[pivot] = t;
        }
        for (long j = i + 1; j < rows; j++) {
            if (d->coeffs[j][i] == 0) continue;
            uint8_t quotient;
            oracle_gf_div(d->coeffs[j][i], d->coeffs[i][i], &quotient);
            for (long k = i; k < cols; k++) d->coeffs[j][k] ^= gf_mul(d->coeffs[i][k], quotient);
            for (size_t k = 0; k < d->plen; k++) d->coded[j][k] ^= gf_mul(d->coded[i][k], quotient);
        }
    }
}

static void ds_clean_backward(oracle_decoder* d) {                     /* :78-134 */
    long rows = (long)d->rows, cols = (long)d->cols;
    long boundary = rows < cols ? rows : cols;
    for (long i = boundary - 1; i >= 0; i--) {
        if (d->coeffs[i][i] == 0) continue;
        for (long j = 0; j < i; j++) {
            if (d->coeffs[j][i] == 0) continue;
            uint8_t quotient;
            oracle_gf_div(d->coeffs[j][i], d->coeffs[i][i], &quotient);
            for (long k = i; k < cols; k++) d->coeffs[j][k] ^= gf_mul(d->coeffs[i][k], quotient);
            for (size_t k = 0; k < d->plen; k++) d->coded[j][k] ^= gf_mul(d->coded[i][k], quotient);
        }
        if (d->coeffs[i][i] == 1) continue;
        uint8_t inv;
        oracle_gf_inv(d->coeffs[i][i], &inv);
        d->coeffs[i][i] = 1;
        for (long j = i + 1; j < cols; j++) {
            if (d->coeffs[i][j] == 0) continue;
            d->coeffs[i][j] = gf_mul(d->coeffs[i][j], inv);
        }
        for (size_t j = 0; j < d->plen; j++) d->coded[i][j] = gf_mul(d->coded[i][j], inv);
    }
}

static void ds_remove_zero_rows(oracle_decoder* d) {                   /* :136-165 */
    for (long i = 0; i < (long)d->rows; i++) {
        int yes = 1;
        for (size_t j = 0; j < d->cols; j++)
            if (d->coeffs[i][j] != 0) { yes = 0; break; }
        if (!yes) continue;
        free(d->coeffs[i]);
        free(d->coded[i]);
        memmove(d->coeffs + i, d->coeffs + i + 1, (d->rows - (size_t)i - 1) * sizeof(uint8_t*));
        memmove(d->coded + i, d->coded + i + 1, (d->rows - (size_t)i - 1) * sizeof(uint8_t*));
        d->rows--;
        i--;
    }
}

void oracle_ds_rref(oracle_decoder* d) {                               /* :178-182 */
    build_tables();
    if (d->rows == 0) return;
    ds_clean_forward(d);
    ds_clean_backward(d);
    ds_remove_zero_rows(d);
}

oracle_decoder* oracle_decoder_new(size_t piece_count) {              /* full/decoder.go:109-112 */
    build_tables();
    oracle_decoder* d = (oracle_decoder*)calloc(1, sizeof(oracle_decoder));
    d->piece_count = piece_count;
    d->expected = piece_count;
    d->cap = piece_count > 0 ? piece_count : 1;
    d->coeffs = (uint8_t**)calloc(d->cap, sizeof(uint8_t*));
    d->coded = (uint8_t**)calloc(d->cap, sizeof(uint8_t*));
    return d;
}

void oracle_decoder_free(oracle_decoder* d) {
    if (!d) return;
    for (size_t i = 0; i < d->rows; i++) { free(d->coeffs[i]); free(d->coded[i]); }
    free(d->coeffs); free(d->coded); free(d);
}

/* decoder_state.go:205-208 (appends copies; kodr aliases the caller's slices) */
static void ds_append(oracle_decoder* d, const uint8_t* vec, size_t vlen, const uint8_t* piece, size_t plen) {
    if (d->rows == d->cap) {
        d->cap *= 2;
        d->coeffs = (uint8_t**)realloc(d->coeffs, d->cap * sizeof(uint8_t*));
        d->coded = (uint8_t**)realloc(d->coded, d->cap * sizeof(uint8_t*));
    }
    if (d->rows == 0) { d->cols = vlen; d->plen = plen; }
    uint8_t* v = (uint8_t*)malloc(vlen ? vlen : 1); memcpy(v, vec, vlen);
    uint8_t* p = (uint8_t*)malloc(plen ? plen : 1); memcpy(p, piece, plen);
    d->coeffs[d->rows] = v;
    d->coded[d->rows] = p;
    d->rows++;
}

/* NewDecoderState(coeffs, coded) (decoder_state.go:269-271) + Rref, for KATs. */
oracle_decoder* oracle_ds_from_matrix(const uint8_t* coeffs, size_t rows, size_t cols,
                                      const uint8_t* coded, size_t plen) {
    oracle_decoder* d = oracle_decoder_new(rows);
    for (size_t i = 0; i < rows; i++) ds_append(d, coeffs + i * cols, cols, coded + i * plen, plen);
    return d;
}

size_t oracle_ds_rows(const oracle_decoder* d) { return d->rows; }     /* Rank :187-189 */
size_t oracle_ds_cols(const oracle_decoder* d) { return d->cols; }
void oracle_ds_coeffs(const oracle_decoder* d, uint8_t* out) {
    for (size_t i = 0; i < d->rows; i++) memcpy(out + i * d->cols, d->coeffs[i], d->cols);
}
void oracle_ds_coded(const oracle_decoder* d, uint8_t* out) {
    for (size_t i = 0; i < d->rows; i++) memcpy(out + i * d->plen, d->coded[i], d->plen);
}

/* full/decoder.go:32-40 */
int oracle_decoder_is_decoded(const oracle_decoder* d) { return d->useful >= d->expected; }
size_t oracle_decoder_required(const oracle_decoder* d) { return d->expected - d->useful; }
size_t oracle_decoder_useful(const oracle_decoder* d) { return d->useful; }
size_t oracle_decoder_received(const oracle_decoder* d) { return d->received; }
/* full/decoder.go:18-25 */
size_t oracle_decoder_piece_length(const oracle_decoder* d) { return d->received > 0 ? d->plen : 0; }

/* full/decoder.go:50-66 */
int oracle_decoder_add_piece(oracle_decoder* d, const uint8_t* vec, size_t vlen,
                             const uint8_t* piece, size_t plen) {
    if (oracle_decoder_is_decoded(d)) return ERR_ALL_USEFUL_RECEIVED;  /* :52-54 */
    ds_append(d, vec, vlen, piece, plen);                              /* :56 */
    d->received++;                                                     /* :57 */
    if (!(d->received > 1)) { d->useful++; return OK; }                /* :58-61 */
    oracle_ds_rref(d);                                                 /* :63 */
    d->useful = d->rows;                                               /* :64 */
    return OK;
}

/* decoder_state.go:221-261 */
int oracle_decoder_get_piece(const oracle_decoder* d, size_t idx, uint8_t* out) {
    if (idx >= d->piece_count) return ERR_PIECE_OUT_OF_BOUND;          /* :222-224 */
    if (idx >= d->rows) return ERR_NOT_DECODED_YET;                    /* :225-227 */
    if (d->rows >= d->piece_count) {                                   /* :229-231 */
        memcpy(out, d->coded[idx], d->plen);
        return OK;
    }
    int decoded = 1;                                                   /* :233-252 */
    for (size_t i = 0; i < d->cols; i++) {
        if (i == idx) {
            if (d->coeffs[idx][i] != 1) { decoded = 0; break; }
        } else {
            if (d->coeffs[idx][i] == 0) { decoded = 0; break; }
        }
    }
    if (!decoded) return ERR_NOT_DECODED_YET;                          /* :254-256 */
    memcpy(out, d->coded[idx], d->plen);                               /* :258-260 */
    return OK;
}

/* full/decoder.go:83-99 */
int oracle_decoder_get_pieces(const oracle_decoder* d, uint8_t* out) {
    if (!oracle_decoder_is_decoded(d)) return ERR_MORE_USEFUL_REQUIRED;
    for (size_t i = 0; i < d->useful; i++) {
        int e = oracle_decoder_get_piece(d, i, out + i * d->plen);
        if (e) return e;
    }
    return OK;
}

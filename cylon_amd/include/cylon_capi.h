/* C ABI of cylon_amd (P8 / J2 base layer).
 *
 * Reference: python/pycylon/api/lib.pyx (Cython C-API wrap/unwrap) and
 * cpp/src/cylon/table_api.hpp + java/src/main/native (JNI over the string-ID
 * table registry).  Every function is exported from the cylon_amd._C shared
 * object with C linkage, so C, C++, JNI or ctypes code can drive the engine
 * without Python: tables live in the process-wide registry under string IDs.
 * Return value: 0 = OK, otherwise a cylon Code (see cylon_amd.Code);
 * cylon_last_error() describes the last failure of the calling thread.
 */
#ifndef CYLON_AMD_CAPI_H_
#define CYLON_AMD_CAPI_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int cylon_capi_version(void);
const char *cylon_last_error(void);

/* context: "cpu" or "cuda:<i>" (local, rank 0 of 1) */
int cylon_init(const char *device);
/* distributed context from the torchrun environment (RANK, WORLD_SIZE, MASTER_ADDR,
   MASTER_PORT, LOCAL_RANK): comm_type "rccl" (one GPU per rank, cuda:<LOCAL_RANK>),
   "tcp" / "gloo" (host tables over the native TCP mesh) or "mpi" (rccl if GPUs are
   visible, else tcp).  Reference: CylonContext::InitDistributed(MPIConfig). */
int cylon_init_distributed(const char *comm_type);
int cylon_get_rank(void);
int cylon_get_world_size(void);
int cylon_barrier(void);
int cylon_finalize(void);

/* tables (string IDs) */
int cylon_read_csv(const char *path, const char *table_id);
int cylon_write_csv(const char *table_id, const char *path);
int64_t cylon_row_count(const char *table_id);
int32_t cylon_column_count(const char *table_id);
int cylon_remove_table(const char *table_id);
/* join_type: 0 inner, 1 left, 2 right, 3 full outer; algorithm: 0 sort, 1 hash */
int cylon_join(const char *left_id, const char *right_id, int join_type, int algorithm, int left_col,
               int right_col, const char *dest_id);
int cylon_distributed_join(const char *left_id, const char *right_id, int join_type, int algorithm, int left_col,
                           int right_col, const char *dest_id);
/* set ops: op 0 union, 1 subtract, 2 intersect */
int cylon_set_op(const char *a_id, const char *b_id, int op, int distributed, const char *dest_id);
int cylon_sort(const char *table_id, int column, int ascending, const char *dest_id);
int cylon_project(const char *table_id, const int32_t *columns, int ncolumns, const char *dest_id);

int cylon_merge(const char *const *table_ids, int ntables, const char *dest_id);
/* print rows [row_begin, row_end) (row_end < 0: all) to stdout, reference Table::Print */
int cylon_print(const char *table_id, int64_t row_begin, int64_t row_end);

/* build a table from host buffers (copied; J1 ArrowTable path).  types: cylon Type numbering
   (INT64 = 8, DOUBLE = 11, STRING = 12, ...); validity: Arrow-style bitmaps (LSB first) or NULL;
   offsets: int32 Arrow offsets for STRING/BINARY columns (NULL otherwise). */
int cylon_table_from_buffers(const char *table_id, int ncols, const char *const *names, const int32_t *types,
                             int64_t nrows, const void *const *data, const uint8_t *const *validity,
                             const int32_t *const *offsets);

/* row predicate selection (reference Table::Select): keep rows for which pred returns non-zero */
typedef struct cylon_row cylon_row;
typedef int (*cylon_row_predicate)(const cylon_row *row, void *user);
int cylon_select(const char *table_id, cylon_row_predicate pred, void *user, const char *dest_id);
int64_t cylon_row_index(const cylon_row *row);
int cylon_row_is_null(const cylon_row *row, int col);
int64_t cylon_row_get_int64(const cylon_row *row, int col);
double cylon_row_get_double(const cylon_row *row, int col);
/* copies up to cap-1 bytes + NUL; returns the full length */
int64_t cylon_row_get_string(const cylon_row *row, int col, char *buf, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif

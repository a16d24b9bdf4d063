/*
 * eks_io.h -- host-side I/O of libeks_hip.so (F1).
 *
 * Replaces the pandas parse of the DLC / Lightning-Pose prediction CSVs in
 * the reference's scripts:
 *   scripts/multicam_example.py:83-92 and scripts/pupil_example.py:63-72
 *   (pd.read_csv(path, header=[0, 1, 2], index_col=0) then
 *   eks/utils.py:13-22 convert_lp_dlc).
 * Plain C ABI, host pointers only.  Returns EKS_IO_OK or an error code with
 * a message in eks_io_last_error().
 */
#ifndef EKS_IO_H
#define EKS_IO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { EKS_IO_OK = 0, EKS_IO_ERR_ARG = 1, EKS_IO_ERR_FILE = 8, EKS_IO_ERR_FORMAT = 16 };

const char *eks_io_last_error(void);

/* Count the data rows (non-blank lines after `header_rows` header lines) and
 * numeric columns (fields per line minus the index field) of a CSV file;
 * *header_bytes = bytes needed for the header text plus NUL. */
int eks_csv_probe(const char *path, int header_rows, int64_t *rows, int64_t *cols,
                  int64_t *header_bytes);

/* Parse the file into data (rows, cols) row-major float64 (empty fields and
 * pandas' default NA strings -> NaN; numbers correctly rounded), the index
 * column into index (rows) or NULL, and copy the header lines verbatim into
 * header (header_bytes >= probe's value) or NULL.  nthreads <= 0: up to 16. */
int eks_csv_read(const char *path, int header_rows, double *data, int64_t rows, int64_t cols,
                 double *index, char *header, int64_t header_bytes, int nthreads);

#ifdef __cplusplus
}
#endif
#endif /* EKS_IO_H */

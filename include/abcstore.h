/* libabcstore — bulk writer of ABC-SMC populations into pyABC's SQLite
 * schema (host code, no GPU).
 *
 * Replaces the per-object SQLAlchemy unit of work of
 * History._save_to_population_db (pyabc/storage/history.py:616-693) and the
 * schema of pyabc/storage/db_model.py:35-127: one prepared INSERT per table,
 * one transaction per population, row ids assigned by SQLite.  The file stays
 * readable by pyABC's own History (tables abc_smc, populations, models,
 * particles, parameters, samples, summary_statistics; summary statistic
 * values are numpy .npy blobs as written by BytesStorage,
 * storage/numpy_bytes_storage.py:6-24).
 *
 * Calls do not touch Python state, so a ctypes caller drops the GIL for the
 * whole write and the generation loop keeps running.
 * Return codes: 0 ok, < 0 error (message: abc_store_last_error()).
 */
#ifndef ABCSTORE_H
#define ABCSTORE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* abc_store_last_error(void);

/* Open (create) the database file and the pyABC schema (db_model.py). */
int abc_store_open(const char* path, void** handle);
int abc_store_close(void* handle);

/* Run one SQL statement without parameters (PRAGMAs, small updates). */
int abc_store_exec(void* handle, const char* sql);

/* One population of one model (history.py:628-688):
 *   populations(abc_smc_id, t, population_end_time, nr_samples, epsilon)
 *   models(population_id, m, name, p_model)
 *   per particle i: particles(model_id, w[i]);
 *     parameters(particle_id, param_names[k], theta[i*d + k]) for k < d;
 *     samples(particle_id, distance[i]);
 *     summary_statistics(sample_id, stat_names[j],
 *                        npy_prefix || bytes of sum_stats[i*S + j]) for j < S
 *     (S = 0: no sum stats stored, History(stores_sum_stats=False)).
 * npy_prefix: the .npy header of a float64 scalar (npy_prefix_len bytes).
 * Strings are NUL-terminated UTF-8.  *population_id receives the row id. */
int abc_store_write_population(void* handle, int64_t abc_smc_id, int64_t t,
                               const char* end_time, int64_t nr_samples,
                               double epsilon, int64_t m,
                               const char* model_name, double p_model,
                               int64_t n, int d, const char* const* param_names,
                               const double* theta, const double* w,
                               const double* distance, int S,
                               const char* const* stat_names,
                               const double* sum_stats,
                               const unsigned char* npy_prefix,
                               int npy_prefix_len, int64_t* population_id);

#ifdef __cplusplus
}
#endif
#endif /* ABCSTORE_H */

// libabcstore: bulk SQLite writer of populations in pyABC's schema.
//
// Reference: pyabc/storage/history.py:616-693 (_save_to_population_db walks
// every particle, parameter, sample and summary statistic as an ORM object
// and commits them in one SQLAlchemy flush: ~2.9 ms per particle at d = 10,
// SURVEY.md §8f) and the tables of pyabc/storage/db_model.py:35-127.  Here:
// one prepared INSERT per table reused for every row, one transaction per
// population, scalar summary statistics encoded as .npy blobs by appending
// the 8 value bytes to a caller-supplied header (the header numpy.save
// writes for a float64 scalar, so BytesStorage reads them back).
//
// The SQLite C API is the system libsqlite3.so.0; the image ships the
// library without its development header, so the few entry points used are
// declared below (stable C API, sqlite.org/c3ref).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/abcstore.h"

extern "C" {
typedef struct sqlite3 sqlite3;
typedef struct sqlite3_stmt sqlite3_stmt;
int sqlite3_open(const char*, sqlite3**);
int sqlite3_close(sqlite3*);
int sqlite3_exec(sqlite3*, const char*, int (*)(void*, int, char**, char**),
                 void*, char**);
int sqlite3_prepare_v2(sqlite3*, const char*, int, sqlite3_stmt**,
                       const char**);
int sqlite3_bind_int64(sqlite3_stmt*, int, long long);
int sqlite3_bind_double(sqlite3_stmt*, int, double);
int sqlite3_bind_text(sqlite3_stmt*, int, const char*, int, void (*)(void*));
int sqlite3_bind_blob(sqlite3_stmt*, int, const void*, int, void (*)(void*));
int sqlite3_step(sqlite3_stmt*);
int sqlite3_reset(sqlite3_stmt*);
int sqlite3_finalize(sqlite3_stmt*);
const char* sqlite3_errmsg(sqlite3*);
void sqlite3_free(void*);
long long sqlite3_last_insert_rowid(sqlite3*);
}

namespace {

constexpr int SQLITE_OK = 0;
constexpr int SQLITE_DONE = 101;
void (*const SQLITE_STATIC)(void*) = nullptr;

thread_local std::string g_err;

int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}

// db_model.py:35-127 as SQLAlchemy emits it for SQLite
const char* kSchema =
    "CREATE TABLE IF NOT EXISTS abc_smc (id INTEGER NOT NULL, start_time "
    "DATETIME, end_time DATETIME, json_parameters VARCHAR(5000), "
    "distance_function VARCHAR(5000), epsilon_function VARCHAR(5000), "
    "population_strategy VARCHAR(5000), git_hash VARCHAR(120), PRIMARY KEY "
    "(id));"
    "CREATE TABLE IF NOT EXISTS populations (id INTEGER NOT NULL, abc_smc_id "
    "INTEGER, t INTEGER, population_end_time DATETIME, nr_samples INTEGER, "
    "epsilon FLOAT, PRIMARY KEY (id), FOREIGN KEY(abc_smc_id) REFERENCES "
    "abc_smc (id));"
    "CREATE TABLE IF NOT EXISTS models (id INTEGER NOT NULL, population_id "
    "INTEGER, m INTEGER, name VARCHAR(200), p_model FLOAT, PRIMARY KEY (id), "
    "FOREIGN KEY(population_id) REFERENCES populations (id));"
    "CREATE TABLE IF NOT EXISTS particles (id INTEGER NOT NULL, model_id "
    "INTEGER, w FLOAT, PRIMARY KEY (id), FOREIGN KEY(model_id) REFERENCES "
    "models (id));"
    "CREATE TABLE IF NOT EXISTS parameters (id INTEGER NOT NULL, particle_id "
    "INTEGER, name VARCHAR(200), value FLOAT, PRIMARY KEY (id), FOREIGN "
    "KEY(particle_id) REFERENCES particles (id));"
    "CREATE TABLE IF NOT EXISTS samples (id INTEGER NOT NULL, particle_id "
    "INTEGER, distance FLOAT, PRIMARY KEY (id), FOREIGN KEY(particle_id) "
    "REFERENCES particles (id));"
    "CREATE TABLE IF NOT EXISTS summary_statistics (id INTEGER NOT NULL, "
    "sample_id INTEGER, name VARCHAR(200), value BLOB, PRIMARY KEY (id), "
    "FOREIGN KEY(sample_id) REFERENCES samples (id));";

struct Store {
  sqlite3* db = nullptr;
};

int exec(sqlite3* db, const char* sql) {
  char* msg = nullptr;
  if (sqlite3_exec(db, sql, nullptr, nullptr, &msg) != SQLITE_OK) {
    std::string m = msg ? msg : "sqlite3_exec failed";
    sqlite3_free(msg);
    return fail(m);
  }
  return 0;
}

// Prepared statements of one population write, finalized on scope exit.
struct Stmts {
  sqlite3* db;
  sqlite3_stmt* s[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  explicit Stmts(sqlite3* d) : db(d) {}
  ~Stmts() {
    for (auto* p : s)
      if (p) sqlite3_finalize(p);
  }
  int prepare() {
    static const char* sql[6] = {
        "INSERT INTO populations (abc_smc_id, t, population_end_time, "
        "nr_samples, epsilon) VALUES (?, ?, ?, ?, ?)",
        "INSERT INTO models (population_id, m, name, p_model) VALUES (?, ?, ?, ?)",
        "INSERT INTO particles (model_id, w) VALUES (?, ?)",
        "INSERT INTO parameters (particle_id, name, value) VALUES (?, ?, ?)",
        "INSERT INTO samples (particle_id, distance) VALUES (?, ?)",
        "INSERT INTO summary_statistics (sample_id, name, value) VALUES (?, ?, ?)"};
    for (int i = 0; i < 6; ++i)
      if (sqlite3_prepare_v2(db, sql[i], -1, &s[i], nullptr) != SQLITE_OK)
        return fail(std::string("prepare: ") + sqlite3_errmsg(db));
    return 0;
  }
};

// step + reset; returns the new row id or -1
long long step(sqlite3* db, sqlite3_stmt* st) {
  if (sqlite3_step(st) != SQLITE_DONE) {
    fail(std::string("insert: ") + sqlite3_errmsg(db));
    sqlite3_reset(st);
    return -1;
  }
  sqlite3_reset(st);
  return sqlite3_last_insert_rowid(db);
}

int write_population(sqlite3* db, int64_t abc_smc_id, int64_t t,
                     const char* end_time, int64_t nr_samples, double epsilon,
                     int64_t m, const char* model_name, double p_model,
                     int64_t n, int d, const char* const* pnames,
                     const double* theta, const double* w,
                     const double* distance, int S, const char* const* snames,
                     const double* ss, const unsigned char* prefix,
                     int prefix_len, int64_t* population_id) {
  Stmts st(db);
  if (st.prepare()) return -1;
  sqlite3_stmt *pop = st.s[0], *mod = st.s[1], *par = st.s[2], *prm = st.s[3],
               *smp = st.s[4], *sst = st.s[5];
  sqlite3_bind_int64(pop, 1, abc_smc_id);
  sqlite3_bind_int64(pop, 2, t);
  sqlite3_bind_text(pop, 3, end_time, -1, SQLITE_STATIC);
  sqlite3_bind_int64(pop, 4, nr_samples);
  sqlite3_bind_double(pop, 5, epsilon);
  const long long pid = step(db, pop);
  if (pid < 0) return -1;
  sqlite3_bind_int64(mod, 1, pid);
  sqlite3_bind_int64(mod, 2, m);
  sqlite3_bind_text(mod, 3, model_name, -1, SQLITE_STATIC);
  sqlite3_bind_double(mod, 4, p_model);
  const long long mid = step(db, mod);
  if (mid < 0) return -1;
  std::vector<unsigned char> blob(prefix_len + 8);
  if (prefix_len) memcpy(blob.data(), prefix, prefix_len);
  sqlite3_bind_int64(par, 1, mid);
  for (int64_t i = 0; i < n; ++i) {
    sqlite3_bind_double(par, 2, w[i]);
    const long long partid = step(db, par);
    if (partid < 0) return -1;
    sqlite3_bind_int64(prm, 1, partid);
    for (int k = 0; k < d; ++k) {
      sqlite3_bind_text(prm, 2, pnames[k], -1, SQLITE_STATIC);
      sqlite3_bind_double(prm, 3, theta[i * d + k]);
      if (step(db, prm) < 0) return -1;
    }
    sqlite3_bind_int64(smp, 1, partid);
    sqlite3_bind_double(smp, 2, distance[i]);
    const long long sid = step(db, smp);
    if (sid < 0) return -1;
    if (S > 0) {
      sqlite3_bind_int64(sst, 1, sid);
      for (int j = 0; j < S; ++j) {
        memcpy(blob.data() + prefix_len, &ss[i * (int64_t)S + j], 8);
        sqlite3_bind_text(sst, 2, snames[j], -1, SQLITE_STATIC);
        sqlite3_bind_blob(sst, 3, blob.data(), (int)blob.size(), SQLITE_STATIC);
        if (step(db, sst) < 0) return -1;
      }
    }
  }
  if (population_id) *population_id = pid;
  return 0;
}

}  // namespace

extern "C" const char* abc_store_last_error(void) { return g_err.c_str(); }

extern "C" int abc_store_open(const char* path, void** handle) {
  if (!path || !handle) return fail("open: null argument");
  Store* s = new Store;
  if (sqlite3_open(path, &s->db) != SQLITE_OK) {
    std::string m = s->db ? sqlite3_errmsg(s->db) : "sqlite3_open failed";
    if (s->db) sqlite3_close(s->db);
    delete s;
    return fail("open: " + m);
  }
  if (exec(s->db, kSchema)) {
    sqlite3_close(s->db);
    delete s;
    return -1;
  }
  *handle = s;
  return 0;
}

extern "C" int abc_store_close(void* handle) {
  Store* s = static_cast<Store*>(handle);
  if (!s) return 0;
  int rc = sqlite3_close(s->db) == SQLITE_OK ? 0 : fail("close: database busy");
  delete s;
  return rc;
}

extern "C" int abc_store_exec(void* handle, const char* sql) {
  Store* s = static_cast<Store*>(handle);
  if (!s || !sql) return fail("exec: null argument");
  return exec(s->db, sql);
}

extern "C" int abc_store_write_population(
    void* handle, int64_t abc_smc_id, int64_t t, const char* end_time,
    int64_t nr_samples, double epsilon, int64_t m, const char* model_name,
    double p_model, int64_t n, int d, const char* const* param_names,
    const double* theta, const double* w, const double* distance, int S,
    const char* const* stat_names, const double* sum_stats,
    const unsigned char* npy_prefix, int npy_prefix_len,
    int64_t* population_id) {
  Store* s = static_cast<Store*>(handle);
  if (!s) return fail("write: null handle");
  if (n < 0 || d < 0 || S < 0 || npy_prefix_len < 0)
    return fail("write: negative size");
  if (n > 0 && (!w || !distance || (d && (!theta || !param_names)) ||
                (S && (!sum_stats || !stat_names))))
    return fail("write: null array");
  if (!end_time || !model_name) return fail("write: null string");
  if (exec(s->db, "BEGIN")) return -1;
  int rc = write_population(s->db, abc_smc_id, t, end_time, nr_samples,
                            epsilon, m, model_name, p_model, n, d, param_names,
                            theta, w, distance, S, stat_names, sum_stats,
                            npy_prefix, npy_prefix_len, population_id);
  if (rc) {
    std::string keep = g_err;
    exec(s->db, "ROLLBACK");
    g_err = keep;
    return -1;
  }
  return exec(s->db, "COMMIT");
}

/*
 * erl_nif.h — a TEST DOUBLE of the documented erl_nif API (OTP 19.3+), just
 * the part integration/c_src/vmqg_nif.c uses, so that the NIF glue is
 * compiled with -Wall -Werror and run by tests/c/nif_mock_check.c
 * (tests/test_nif_layer.py).  OTP is not in this image; this is not the OTP
 * header and not a runtime: terms are immutable heap cells (see
 * erl_nif_mock.c), environments never free them, dirty-scheduler flags are
 * accepted and ignored (the check calls the NIFs from plain threads).
 */
#ifndef MOCK_ERL_NIF_H
#define MOCK_ERL_NIF_H

#include <stddef.h>
#include <stdint.h>

typedef uintptr_t ERL_NIF_TERM;
typedef struct enif_environment_t ErlNifEnv;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef void ErlNifResourceDtor(ErlNifEnv*, void*);

typedef struct {
  size_t size;
  unsigned char* data;
  void* ref_bin;   /* mock: owned buffer to free on release */
} ErlNifBinary;

typedef struct {
  const char* name;
  unsigned arity;
  ERL_NIF_TERM (*fptr)(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]);
  unsigned flags;
} ErlNifFunc;

typedef enum { ERL_NIF_LATIN1 = 1 } ErlNifCharEncoding;
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
#define ERL_NIF_DIRTY_JOB_IO_BOUND 1
#define ERL_NIF_DIRTY_JOB_CPU_BOUND 2

typedef struct {
  const char* name;
  int num_of_funcs;
  ErlNifFunc* funcs;
  int (*load)(ErlNifEnv*, void**, ERL_NIF_TERM);
} ErlNifEntry;

#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                              \
  ErlNifEntry* nif_init(void) {                                                               \
    static ErlNifEntry e = {#NAME, (int)(sizeof(FUNCS) / sizeof((FUNCS)[0])), FUNCS, LOAD};   \
    (void)(RELOAD); (void)(UPGRADE); (void)(UNLOAD);                                          \
    return &e;                                                                                \
  }

typedef struct {
  int driver_major_version, driver_minor_version;
  char* erts_version;
  char* otp_release;
  int thread_support, smp_support, async_threads, scheduler_threads, nif_major_version, nif_minor_version;
  int dirty_scheduler_support;
} ErlNifSysInfo;
void enif_system_info(ErlNifSysInfo* sip, size_t si_size);
/* mock: runs fp at once on the calling thread (no scheduler to hand it to) */
ERL_NIF_TERM enif_schedule_nif(ErlNifEnv* env, const char* fun_name, int flags,
                               ERL_NIF_TERM (*fp)(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]), int argc,
                               const ERL_NIF_TERM argv[]);

/* memory */
void* enif_alloc(size_t size);
void* enif_realloc(void* ptr, size_t size);
void enif_free(void* ptr);
ErlNifEnv* enif_alloc_env(void);
void enif_free_env(ErlNifEnv* env);

/* term construction */
ERL_NIF_TERM enif_make_atom(ErlNifEnv* env, const char* name);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b);
ERL_NIF_TERM enif_make_tuple4(ErlNifEnv* env, ERL_NIF_TERM a, ERL_NIF_TERM b, ERL_NIF_TERM c, ERL_NIF_TERM d);
ERL_NIF_TERM enif_make_list_from_array(ErlNifEnv* env, const ERL_NIF_TERM arr[], unsigned cnt);
ERL_NIF_TERM enif_make_string(ErlNifEnv* env, const char* string, ErlNifCharEncoding encoding);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv* env, uint64_t i);
ERL_NIF_TERM enif_make_uint(ErlNifEnv* env, unsigned i);
ERL_NIF_TERM enif_make_tuple_from_array(ErlNifEnv* env, const ERL_NIF_TERM arr[], unsigned cnt);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv* env);
ERL_NIF_TERM enif_make_copy(ErlNifEnv* dst_env, ERL_NIF_TERM src_term);
ERL_NIF_TERM enif_make_resource(ErlNifEnv* env, void* obj);

/* term inspection */
typedef int64_t ErlNifSInt64;
int enif_get_int(ErlNifEnv* env, ERL_NIF_TERM term, int* ip);
int enif_get_int64(ErlNifEnv* env, ERL_NIF_TERM term, ErlNifSInt64* ip);
/* bytes written including the NUL, 0 if not an atom or it does not fit */
int enif_get_atom(ErlNifEnv* env, ERL_NIF_TERM atom, char* buf, unsigned size, ErlNifCharEncoding encoding);
int enif_get_uint(ErlNifEnv* env, ERL_NIF_TERM term, unsigned* ip);
int enif_get_tuple(ErlNifEnv* env, ERL_NIF_TERM term, int* arity, const ERL_NIF_TERM** array);
int enif_get_list_length(ErlNifEnv* env, ERL_NIF_TERM term, unsigned* len);
int enif_get_list_cell(ErlNifEnv* env, ERL_NIF_TERM list, ERL_NIF_TERM* head, ERL_NIF_TERM* tail);
int enif_get_map_value(ErlNifEnv* env, ERL_NIF_TERM map, ERL_NIF_TERM key, ERL_NIF_TERM* value);
int enif_inspect_binary(ErlNifEnv* env, ERL_NIF_TERM bin_term, ErlNifBinary* bin);
int enif_inspect_iolist_as_binary(ErlNifEnv* env, ERL_NIF_TERM term, ErlNifBinary* bin);
int enif_is_identical(ERL_NIF_TERM lhs, ERL_NIF_TERM rhs);
int enif_term_to_binary(ErlNifEnv* env, ERL_NIF_TERM term, ErlNifBinary* bin);
void enif_release_binary(ErlNifBinary* bin);

/* threads (erl_drv / erl_nif mutexes) */
typedef struct enif_mutex_t ErlNifMutex;
ErlNifMutex* enif_mutex_create(char* name);
void enif_mutex_destroy(ErlNifMutex* mtx);
void enif_mutex_lock(ErlNifMutex* mtx);
void enif_mutex_unlock(ErlNifMutex* mtx);

/* resources */
ErlNifResourceType* enif_open_resource_type(ErlNifEnv* env, const char* module_str, const char* name,
                                            ErlNifResourceDtor* dtor, ErlNifResourceFlags flags,
                                            ErlNifResourceFlags* tried);
void* enif_alloc_resource(ErlNifResourceType* type, size_t size);
void enif_release_resource(void* obj);
void enif_keep_resource(void* obj);
int enif_get_resource(ErlNifEnv* env, ERL_NIF_TERM term, ErlNifResourceType* type, void** objp);

#endif /* MOCK_ERL_NIF_H */

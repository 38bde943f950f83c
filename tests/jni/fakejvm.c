/*
 * fakejvm.c — a functional stand-in for the JNIEnv of a JVM, for the tests only (VERDICT r4 "do this"
 * #3: execute the JNI shim). It implements every JNI function integration/jni/mpi_HipIntracomm.c calls
 * (the table of tests/jni/jni.h) over plain host memory, so the shim can be loaded and driven from
 * ctypes on the GPU box, as a JVM would drive it:
 *   - Java arrays: fj_array() objects with a length in elements and an element size; direct buffers:
 *     fj_direct() objects around caller memory with a capacity in bytes;
 *   - GetPrimitiveArrayCritical returns the elements in place, or — fj_copy_mode(1) — a copy, as a JVM
 *     may: then ReleasePrimitiveArrayCritical's mode decides (0 copy back + free, JNI_COMMIT copy back,
 *     JNI_ABORT free), so a wrong write-back mode in the shim loses or leaks results visibly; several
 *     threads may hold one array at once (legal JNI): each hold gets its own copy;
 *   - ThrowNew leaves a pending exception per thread (fj_exception reads and clears it);
 *   - the JNI rules the shim must keep are checked and counted as violations (fj_violations): any JNI
 *     call other than Get/ReleasePrimitiveArrayCritical while the calling thread holds a critical region
 *     (JNI spec, GetPrimitiveArrayCritical), a release that does not match a get, a region still held
 *     when the native method returns (fj_crit_held), array region calls out of bounds (these also leave
 *     ArrayIndexOutOfBoundsException pending, as the JVM does).
 * Not a JVM and not JDK text: the layout of the function table is tests/jni/jni.h's own.
 */
#include <jni.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define JNI_COMMIT 1

enum { K_CLASS = 1, K_ARRAY = 2, K_DIRECT = 3, K_OBJECT = 4 };
#define FJ_MAX_HOLDS 64

struct _jobject {
  int kind;
  char name[64];   /* K_CLASS */
  char *data;      /* K_ARRAY: elements; K_DIRECT: caller memory */
  long long len;   /* K_ARRAY: elements; K_DIRECT: capacity in bytes */
  int esz;         /* K_ARRAY: bytes per element */
  char *crit_copies[FJ_MAX_HOLDS]; /* copies handed out by GetPrimitiveArrayCritical in copy mode */
  int crit_refs;
  int rel_modes[3]; /* releases seen with mode 0, JNI_COMMIT, JNI_ABORT */
};

static __thread int tl_crit;            /* critical regions this thread holds */
static __thread char tl_exc_class[64];  /* pending exception ("" = none) */
static __thread char tl_exc_msg[1024];
static int g_copy_mode;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_violations;
static char g_vlog[4096];

static void vlog_locked(const char *line) { /* caller holds g_mu */
  g_violations++;
  size_t n = strlen(g_vlog);
  if (n + strlen(line) + 2 < sizeof g_vlog) {
    strcat(g_vlog, line);
    strcat(g_vlog, "\n");
  }
}

static void violation(const char *fmt, ...) {
  char line[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(line, sizeof line, fmt, ap);
  va_end(ap);
  pthread_mutex_lock(&g_mu);
  vlog_locked(line);
  pthread_mutex_unlock(&g_mu);
}

static void no_crit(const char *fn) {
  if (tl_crit > 0) violation("%s called inside a critical region (%d held)", fn, tl_crit);
}

static void throw_pending(const char *cls, const char *msg) {
  if (tl_exc_class[0]) return; /* the first exception stays pending */
  snprintf(tl_exc_class, sizeof tl_exc_class, "%s", cls);
  snprintf(tl_exc_msg, sizeof tl_exc_msg, "%s", msg);
}

static int is_array(jobject o, const char *fn) {
  if (!o || o->kind != K_ARRAY) {
    violation("%s on a non-array object", fn);
    return 0;
  }
  return 1;
}

/* ---- the JNI functions ---- */
static jclass f_FindClass(JNIEnv *env, const char *name) {
  (void)env;
  no_crit("FindClass");
  jobject c = (jobject)calloc(1, sizeof *c);
  c->kind = K_CLASS;
  snprintf(c->name, sizeof c->name, "%s", name);
  return c; /* leaked, as local references are until the native method returns */
}

static jint f_ThrowNew(JNIEnv *env, jclass cls, const char *msg) {
  (void)env;
  no_crit("ThrowNew");
  if (!cls || cls->kind != K_CLASS) {
    violation("ThrowNew without a class");
    return -1;
  }
  throw_pending(cls->name, msg ? msg : "");
  return 0;
}

static jboolean f_ExceptionCheck(JNIEnv *env) {
  (void)env;
  no_crit("ExceptionCheck");
  return tl_exc_class[0] != 0;
}

static jsize f_GetArrayLength(JNIEnv *env, jarray a) {
  (void)env;
  no_crit("GetArrayLength");
  return is_array(a, "GetArrayLength") ? (jsize)a->len : 0;
}

static int region_ok(jarray a, jsize start, jsize len, int esz, const char *fn) {
  if (!is_array(a, fn)) return 0;
  if (a->esz != esz) violation("%s on an array of %d-byte elements", fn, a->esz);
  if (start < 0 || len < 0 || (long long)start + len > a->len) {
    violation("%s out of bounds: [%d, %d) of %lld", fn, start, start + len, a->len);
    throw_pending("java/lang/ArrayIndexOutOfBoundsException", fn);
    return 0;
  }
  return 1;
}

static void f_GetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize start, jsize len, jbyte *buf) {
  (void)env;
  no_crit("GetByteArrayRegion");
  if (region_ok(a, start, len, 1, "GetByteArrayRegion")) memcpy(buf, a->data + start, (size_t)len);
}

static void f_SetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize start, jsize len, const jbyte *buf) {
  (void)env;
  no_crit("SetByteArrayRegion");
  if (region_ok(a, start, len, 1, "SetByteArrayRegion")) memcpy(a->data + start, buf, (size_t)len);
}

static void f_GetIntArrayRegion(JNIEnv *env, jintArray a, jsize start, jsize len, jint *buf) {
  (void)env;
  no_crit("GetIntArrayRegion");
  if (region_ok(a, start, len, 4, "GetIntArrayRegion")) memcpy(buf, a->data + 4 * (size_t)start, 4 * (size_t)len);
}

static jint *f_GetIntArrayElements(JNIEnv *env, jintArray a, jboolean *is_copy) {
  (void)env;
  no_crit("GetIntArrayElements");
  if (!is_array(a, "GetIntArrayElements")) return NULL;
  jint *c = (jint *)malloc(4 * (size_t)(a->len ? a->len : 1)); /* always a copy */
  memcpy(c, a->data, 4 * (size_t)a->len);
  if (is_copy) *is_copy = 1;
  return c;
}

static void f_ReleaseIntArrayElements(JNIEnv *env, jintArray a, jint *elems, jint mode) {
  (void)env;
  no_crit("ReleaseIntArrayElements");
  if (!is_array(a, "ReleaseIntArrayElements") || !elems) return;
  if (mode == 0 || mode == JNI_COMMIT) memcpy(a->data, elems, 4 * (size_t)a->len);
  if (mode != JNI_COMMIT) free(elems);
}

static void *f_GetPrimitiveArrayCritical(JNIEnv *env, jarray a, jboolean *is_copy) {
  (void)env;
  if (!is_array(a, "GetPrimitiveArrayCritical")) return NULL;
  tl_crit++;
  pthread_mutex_lock(&g_mu);
  a->crit_refs++;
  void *p = a->data;
  if (g_copy_mode) {
    int slot = 0;
    while (slot < FJ_MAX_HOLDS && a->crit_copies[slot]) slot++;
    if (slot == FJ_MAX_HOLDS) {
      vlog_locked("GetPrimitiveArrayCritical: more concurrent holds of one array than the stand-in keeps");
      p = NULL;
    } else {
      p = a->crit_copies[slot] = (char *)malloc((size_t)(a->len * a->esz) + 1);
      memcpy(p, a->data, (size_t)(a->len * a->esz));
    }
  }
  pthread_mutex_unlock(&g_mu);
  if (is_copy) *is_copy = g_copy_mode != 0;
  return p;
}

static void f_ReleasePrimitiveArrayCritical(JNIEnv *env, jarray a, void *c, jint mode) {
  (void)env;
  if (!is_array(a, "ReleasePrimitiveArrayCritical")) return;
  if (tl_crit <= 0) violation("ReleasePrimitiveArrayCritical without a matching get");
  tl_crit--;
  pthread_mutex_lock(&g_mu);
  a->crit_refs--;
  if (mode >= 0 && mode <= 2) a->rel_modes[mode]++;
  if (g_copy_mode) {
    int slot = 0;
    while (slot < FJ_MAX_HOLDS && (!c || a->crit_copies[slot] != c)) slot++;
    if (slot == FJ_MAX_HOLDS) {
      vlog_locked("ReleasePrimitiveArrayCritical: not the pointer the get returned");
    } else {
      if (mode == 0 || mode == JNI_COMMIT) memcpy(a->data, c, (size_t)(a->len * a->esz));
      if (mode != JNI_COMMIT) {
        free(a->crit_copies[slot]);
        a->crit_copies[slot] = NULL;
      }
    }
  } else if (c != a->data) {
    vlog_locked("ReleasePrimitiveArrayCritical: not the pointer the get returned");
  }
  pthread_mutex_unlock(&g_mu);
}

static void *f_GetDirectBufferAddress(JNIEnv *env, jobject b) {
  (void)env;
  no_crit("GetDirectBufferAddress");
  return b && b->kind == K_DIRECT ? b->data : NULL;
}

static jlong f_GetDirectBufferCapacity(JNIEnv *env, jobject b) {
  (void)env;
  no_crit("GetDirectBufferCapacity");
  return b && b->kind == K_DIRECT ? (jlong)b->len : -1;
}

static const struct JNINativeInterface_ g_table = {
    f_FindClass,          f_ThrowNew,           f_ExceptionCheck,
    f_GetArrayLength,     f_GetByteArrayRegion, f_SetByteArrayRegion,
    f_GetIntArrayRegion,  f_GetIntArrayElements, f_ReleaseIntArrayElements,
    f_GetPrimitiveArrayCritical, f_ReleasePrimitiveArrayCritical,
    f_GetDirectBufferAddress, f_GetDirectBufferCapacity,
};
static JNIEnv g_env = &g_table;

/* ---- the test driver's side (ctypes) ---- */
JNIEnv *fj_env(void) { return &g_env; }

jobject fj_array(int esz, long long len) {
  jobject o = (jobject)calloc(1, sizeof *o);
  o->kind = K_ARRAY;
  o->esz = esz;
  o->len = len;
  o->data = (char *)calloc((size_t)(len * esz) + 1, 1);
  return o;
}

jobject fj_direct(void *addr, long long capacity) {
  jobject o = (jobject)calloc(1, sizeof *o);
  o->kind = K_DIRECT;
  o->data = (char *)addr;
  o->len = capacity;
  return o;
}

jobject fj_object(void) {
  jobject o = (jobject)calloc(1, sizeof *o);
  o->kind = K_OBJECT;
  return o;
}

void *fj_data(jobject o) { return o ? o->data : NULL; }

void fj_free(jobject o) {
  if (!o) return;
  if (o->kind == K_ARRAY) {
    if (o->crit_refs) violation("array freed while pinned");
    free(o->data);
    for (int i = 0; i < FJ_MAX_HOLDS; i++) free(o->crit_copies[i]);
  }
  free(o);
}

void fj_copy_mode(int on) { g_copy_mode = on; }

/* the calling thread's pending exception: 1 and its class and message (then cleared), or 0 */
int fj_exception(char *cls, int ccap, char *msg, int mcap) {
  if (!tl_exc_class[0]) return 0;
  snprintf(cls, (size_t)ccap, "%s", tl_exc_class);
  snprintf(msg, (size_t)mcap, "%s", tl_exc_msg);
  tl_exc_class[0] = 0;
  tl_exc_msg[0] = 0;
  return 1;
}

/* violations since the last call (their log into buf), then reset */
int fj_violations(char *buf, int cap) {
  pthread_mutex_lock(&g_mu);
  int n = g_violations;
  snprintf(buf, (size_t)cap, "%s", g_vlog);
  g_violations = 0;
  g_vlog[0] = 0;
  pthread_mutex_unlock(&g_mu);
  return n;
}

int fj_crit_held(void) { return tl_crit; }

void fj_release_modes(jobject a, int out[3]) {
  for (int i = 0; i < 3; i++) out[i] = a ? a->rel_modes[i] : 0;
}

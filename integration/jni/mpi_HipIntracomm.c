/*
 * mpi_HipIntracomm.c — JNI shim between mpi.HipIntracomm (integration/java/mpi/HipIntracomm.java)
 * and libmpjx (include/mpjx.h). New code for a maintainer to build where a JDK exists:
 *
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I<repo>/include \
 *       mpi_HipIntracomm.c -L<repo>/mpjexpress_amd/lib -lmpjx -lpthread -Wl,-rpath,<repo>/mpjexpress_amd/lib \
 *       -o libmpjx_jni.so
 *
 * It replaces the body of Java_mpjdev_natmpjdev_Intracomm_nativeReduce
 * (src/mpjdev/natmpjdev/lib/mpjdev_natmpjdev_Intracomm.c:410-627): instead of
 * Get<Type>ArrayElements + MPI_Reduce + one JNI upcall per result element, the Java arrays reach
 * the mpjx_*_host entry points as plain pointers (offset applied here, counts widened to int64):
 * pinned with GetPrimitiveArrayCritical when this JVM holds one rank, copied in and out under short
 * critical sections in multicore mode (see hbuf). Status codes become mpi.MPIException
 * (src/mpi/MPIException.java:42) carrying mpjx_last_error(), where the reference ignored MPI's
 * return code.
 *
 * The build image has no JDK: the repository compiles this file against the subset of jni.h it uses
 * (tests/jni/jni.h) and runs it against a functional stand-in JNIEnv (tests/jni/fakejvm.c,
 * tests/test_jni_fake.py and tests/test_gpu_jni.py); a maintainer builds it as above.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpjx.h"

static int throw_mpi(JNIEnv *env, int status, const char *what) {
  char msg[640];
  snprintf(msg, sizeof msg, "%s: %s: %s", what, mpjx_strerror(status), mpjx_last_error());
  jclass ex = (*env)->FindClass(env, "mpi/MPIException");
  if (ex) (*env)->ThrowNew(env, ex, msg);
  return status;
}

/* The 128-byte world id from a Java byte[]: 0 (with an exception pending) if it is shorter. */
static int get_id(JNIEnv *env, jbyteArray arr, mpjx_unique_id *id) {
  if (!arr || (*env)->GetArrayLength(env, arr) < (jsize)sizeof *id) {
    throw_mpi(env, MPJX_ERR_ARG, "world id: a byte[] of at least 128 bytes is required");
    return 0;
  }
  (*env)->GetByteArrayRegion(env, arr, 0, (jsize)sizeof *id, (jbyte *)id);
  return !(*env)->ExceptionCheck(env);
}

JNIEXPORT jint JNICALL Java_mpi_HipIntracomm_nativeDeviceCount(JNIEnv *env, jclass cls) {
  int n = 0;
  (void)cls;
  int rc = mpjx_device_count(&n);
  if (rc) throw_mpi(env, rc, "mpjx_device_count");
  return n;
}

JNIEXPORT void JNICALL Java_mpi_HipIntracomm_nativeUniqueId(JNIEnv *env, jclass cls, jbyteArray uid) {
  mpjx_unique_id id;
  (void)cls;
  int rc = mpjx_get_unique_id(&id);
  if (rc) { throw_mpi(env, rc, "mpjx_get_unique_id"); return; }
  (*env)->SetByteArrayRegion(env, uid, 0, (jsize)sizeof id, (const jbyte *)&id);
}

JNIEXPORT jlong JNICALL Java_mpi_HipIntracomm_nativeInitRank(JNIEnv *env, jclass cls, jint rank, jint size,
                                                             jint device, jbyteArray uid) {
  mpjx_unique_id id;
  mpjx_comm_t c = NULL;
  (void)cls;
  if (!get_id(env, uid, &id)) return 0;
  int rc = mpjx_comm_init_rank(&c, size, &id, rank, device);
  if (rc) { throw_mpi(env, rc, "mpjx_comm_init_rank"); return 0; }
  return (jlong)(intptr_t)c;
}

/* several JVMs of one node without RCCL: the HIP-IPC direct engine (id: any 128 bytes per world) */
JNIEXPORT jlong JNICALL Java_mpi_HipIntracomm_nativeInitIpc(JNIEnv *env, jclass cls, jint rank, jint size,
                                                            jint device, jbyteArray uid) {
  mpjx_unique_id id;
  mpjx_comm_t c = NULL;
  (void)cls;
  if (!get_id(env, uid, &id)) return 0;
  int rc = mpjx_comm_init_ipc(&c, size, &id, rank, device);
  if (rc) { throw_mpi(env, rc, "mpjx_comm_init_ipc"); return 0; }
  return (jlong)(intptr_t)c;
}

/* multicore (smpdev): each rank thread forms its communicator's world itself; libmpjx's process-wide
 * registry (mpjx_comm_init_smp_rank) hands every thread its handle, whichever shim copy it called
 * through. One world per communicator (COMM_WORLD, every Split/Create), keyed by the id rank 0 drew. */
static volatile int g_multicore = 0; /* the ranks are threads of this JVM (set by nativeInitSmp) */

JNIEXPORT jlong JNICALL Java_mpi_HipIntracomm_nativeInitSmp(JNIEnv *env, jclass cls, jbyteArray id, jint rank,
                                                            jint size, jintArray devices) {
  mpjx_unique_id uid;
  mpjx_comm_t c = NULL;
  (void)cls;
  if (size < 1 || (*env)->GetArrayLength(env, devices) < size) {
    throw_mpi(env, MPJX_ERR_ARG, "nativeInitSmp: devices[] shorter than the communicator");
    return 0;
  }
  if (!get_id(env, id, &uid)) return 0;
  int *devs = (int *)calloc((size_t)size, sizeof(int));
  if (!devs) {
    throw_mpi(env, MPJX_ERR_ARG, "nativeInitSmp: out of memory");
    return 0;
  }
  (*env)->GetIntArrayRegion(env, devices, 0, size, (jint *)devs);
  if ((*env)->ExceptionCheck(env)) { /* pending ArrayIndexOutOfBoundsException: leave it to Java */
    free(devs);
    return 0;
  }
  int rc = mpjx_comm_init_smp_rank(&c, size, &uid, rank, devs);
  free(devs);
  if (rc) { throw_mpi(env, rc, "mpjx_comm_init_smp_rank"); return 0; }
  g_multicore = 1;
  return (jlong)(intptr_t)c;
}

static void stage_release(void);

JNIEXPORT void JNICALL Java_mpi_HipIntracomm_nativeFree(JNIEnv *env, jclass cls, jlong comm) {
  (void)cls;
  int rc = mpjx_comm_destroy((mpjx_comm_t)(intptr_t)comm);
  stage_release(); /* this rank thread's page-locked staging (Finalize frees COMM_WORLD last) */
  if (rc) throw_mpi(env, rc, "mpjx_comm_destroy");
}

/* Buffers handed to libmpjx. A direct ByteBuffer (mpjbuf NIOBuffer) is used in place. A Java array
 * is pinned with GetPrimitiveArrayCritical for the whole call when this JVM holds one rank: the call
 * then waits only on other processes. In multicore mode the rank threads of this JVM wait for each
 * other inside every call, and a thread inside a critical region holds up garbage collection: a rank
 * thread that must allocate on its way to the collective would never arrive. There the array is
 * copied in and out under short critical sections instead (two host memcpy's of the payload).
 * JNI forbids every other JNI call while a critical region is held, so a call first classifies and
 * bounds-checks ALL its buffers (hb_prepare: GetDirectBufferAddress/Capacity, GetArrayLength) and
 * only then pins them (hb_pin); the releases (hb_close) come before any exception is raised. A buffer
 * that fails its check reaches libmpjx as NULL: libmpjx rejects the call and, in multicore and IPC
 * worlds, releases the other ranks instead of letting them wait for this one; the shim's own message
 * is then the exception's. */
typedef struct {
  jarray arr;  /* the Java array, or NULL (direct buffer / no buffer) */
  void *crit;  /* array elements pinned across the call, or NULL */
  char *copy;  /* the copy (multicore mode): this thread's page-locked staging, or malloc'd; or NULL */
  int owned;   /* copy is malloc'd (freed on close), not the thread's staging */
  char *data;  /* what libmpjx reads / writes; NULL if the checks or the copy failed */
  size_t off, bytes;
} hbuf;

/* 1 if `buf` (may be NULL: no buffer) holds [offset, offset + count) elements of `type`; else 0 with
 * the reason in err[]. Offsets are Java array indices, i.e. base elements (half a pair for the *2
 * types), as in NativeIntracomm (src/mpi/NativeIntracomm.java:1072-1115). */
static int hb_prepare(JNIEnv *env, jobject buf, int elem_offset, int type, int64_t count, hbuf *h, char *err,
                      size_t errlen, const char *what) {
  memset(h, 0, sizeof *h);
  const size_t base = (size_t)mpjx_type_size(type & 0xff);
  h->bytes = count > 0 ? (size_t)count * (size_t)mpjx_type_size(type) : 0;
  if (!buf) return 1;
  if (elem_offset < 0 || base == 0) {
    snprintf(err, errlen, "%s: offset %d or datatype %d invalid", what, elem_offset, type);
    return 0;
  }
  h->off = (size_t)elem_offset * base;
  char *addr = (char *)(*env)->GetDirectBufferAddress(env, buf);
  if (addr) {
    /* a direct ByteBuffer (mpjbuf's NIOBuffer): its capacity, in elements per the JNI spec, is bytes.
     * A typed view (asDoubleBuffer()) would report elements and fail this check conservatively. */
    const jlong cap = (*env)->GetDirectBufferCapacity(env, buf);
    if (cap >= 0 && h->off + h->bytes > (size_t)cap) {
      snprintf(err, errlen, "%s: direct buffer of %lld bytes is too small for %zu bytes at byte offset %zu", what,
               (long long)cap, h->bytes, h->off);
      return 0;
    }
    h->data = addr + h->off;
    return 1;
  }
  h->arr = (jarray)buf;
  const jsize len = (*env)->GetArrayLength(env, h->arr);
  if (h->off + h->bytes > (size_t)len * base) {
    snprintf(err, errlen, "%s: array of %d elements is too short for offset %d + %lld x %d-byte elements", what,
             (int)len, elem_offset, (long long)count, mpjx_type_size(type));
    h->arr = NULL;
    return 0;
  }
  return 1;
}

/* Multicore mode copies through page-locked staging kept per rank thread (two regions: send, recv),
 * allocated by libmpjx (mpjx_host_alloc) and grown on demand: the *_host calls then take their
 * host-direct form (no device staging; include/mpjx.h). The regions belong to the thread: a pthread key's
 * destructor frees them when the rank thread exits, and nativeFree frees the calling thread's (a JVM's
 * rank threads outlive their communicators). A region larger than the cap (MPJX_JNI_STAGE_CAP_MIB,
 * default 64 MiB; above one host-pipeline chunk the host-direct form does not apply anyway) is not kept:
 * such calls copy through malloc'd memory freed with the call. malloc'd copies too if the page-locked
 * allocation fails. mpjx_jni_staging_live() counts the regions alive in the process (diagnostic). */
#include <pthread.h>
#include <stdatomic.h>

typedef struct {
  void *p[2];
  size_t bytes[2];
} stage_t;

static pthread_key_t g_stage_key;
static pthread_once_t g_stage_once = PTHREAD_ONCE_INIT;
static atomic_long g_stage_live;

static void stage_free(void *v) {
  stage_t *st = (stage_t *)v;
  if (!st) return;
  for (int i = 0; i < 2; i++)
    if (st->p[i]) {
      mpjx_host_free(st->p[i]);
      atomic_fetch_sub(&g_stage_live, 1);
    }
  free(st);
}

static void stage_key_init(void) { (void)pthread_key_create(&g_stage_key, stage_free); }

static stage_t *stage_tls(int create) {
  (void)pthread_once(&g_stage_once, stage_key_init);
  stage_t *st = (stage_t *)pthread_getspecific(g_stage_key);
  if (!st && create) {
    st = (stage_t *)calloc(1, sizeof *st);
    if (st && pthread_setspecific(g_stage_key, st) != 0) {
      free(st);
      st = NULL;
    }
  }
  return st;
}

static size_t stage_cap(void) {
  const char *e = getenv("MPJX_JNI_STAGE_CAP_MIB");
  const long m = e ? atol(e) : 64;
  return (size_t)(m > 0 ? m : 64) << 20;
}

long mpjx_jni_staging_live(void);
long mpjx_jni_staging_live(void) { return atomic_load(&g_stage_live); }

static char *stage_get(int which, size_t bytes) {
  if (bytes > stage_cap()) return NULL;
  stage_t *st = stage_tls(1);
  if (!st) return NULL;
  if (st->bytes[which] < bytes || !st->p[which]) {
    size_t want = bytes > 2 * st->bytes[which] ? bytes : 2 * st->bytes[which];
    if (want > stage_cap()) want = stage_cap();
    void *p = NULL;
    if (mpjx_host_alloc(&p, (int64_t)want) != MPJX_SUCCESS || !p) return NULL;
    if (st->p[which]) {
      mpjx_host_free(st->p[which]);
    } else {
      atomic_fetch_add(&g_stage_live, 1);
    }
    st->p[which] = p;
    st->bytes[which] = want;
  }
  return (char *)st->p[which];
}

/* Frees the calling thread's staging; the next multicore call allocates it again. */
static void stage_release(void) {
  stage_t *st = stage_tls(0);
  if (!st) return;
  (void)pthread_setspecific(g_stage_key, NULL);
  stage_free(st);
}

/* Pins (or, multicore, copies in) a prepared array; direct buffers and absent buffers are ready.
 * which: 0 send, 1 recv (the thread's staging region). */
static void hb_pin(JNIEnv *env, hbuf *h, int copy_in, int which) {
  if (!h->arr) return;
  if (!g_multicore) {
    h->crit = (*env)->GetPrimitiveArrayCritical(env, h->arr, NULL);
    h->data = h->crit ? (char *)h->crit + h->off : NULL;
    return;
  }
  h->copy = stage_get(which, h->bytes ? h->bytes : 1);
  if (!h->copy) {
    h->copy = (char *)malloc(h->bytes ? h->bytes : 1);
    h->owned = 1;
  }
  if (h->copy && copy_in && h->bytes) {
    char *a = (char *)(*env)->GetPrimitiveArrayCritical(env, h->arr, NULL);
    if (a) {
      memcpy(h->copy, a + h->off, h->bytes);
      (*env)->ReleasePrimitiveArrayCritical(env, h->arr, a, JNI_ABORT);
    } else {
      if (h->owned) free(h->copy);
      h->copy = NULL;
    }
  }
  h->data = h->copy;
}

/* write_back: the call succeeded and wrote this buffer (mode 0: copy back and release); otherwise the
 * Java array is left as it was (JNI_ABORT). */
static void hb_close(JNIEnv *env, hbuf *h, int write_back) {
  if (h->crit) (*env)->ReleasePrimitiveArrayCritical(env, h->arr, h->crit, write_back ? 0 : JNI_ABORT);
  if (h->copy) {
    if (write_back && h->bytes) {
      char *a = (char *)(*env)->GetPrimitiveArrayCritical(env, h->arr, NULL);
      if (a) {
        memcpy(a + h->off, h->copy, h->bytes);
        (*env)->ReleasePrimitiveArrayCritical(env, h->arr, a, 0);
      }
    }
    if (h->owned) free(h->copy);
  }
  memset(h, 0, sizeof *h);
}

/* The status of a call, raised as mpi.MPIException after every buffer is released: the shim's own
 * argument check first (err[]), else libmpjx's. */
static void raise_status(JNIEnv *env, int rc, const char *err, const char *what) {
  if (!rc) return;
  if (err[0]) {
    jclass ex = (*env)->FindClass(env, "mpi/MPIException");
    if (ex) (*env)->ThrowNew(env, ex, err);
    return;
  }
  throw_mpi(env, rc, what);
}

#define COMM(c) ((mpjx_comm_t)(intptr_t)(c))

JNIEXPORT void JNICALL Java_mpi_HipIntracomm_nativeReduce(JNIEnv *env, jobject self, jlong comm, jobject send,
                                                          jint soff, jobject recv, jint roff, jint count,
                                                          jint type, jint op, jint root, jint flags) {
  (void)self;
  hbuf hs, hr;
  char err[256] = "";
  int me = -1;
  mpjx_comm_rank(COMM(comm), &me);
  /* recvbuf: significant at the root; under MPJX_FLAG_FAITHFUL every rank's is written (the MST
   * sub-tree partial / FT send copy PureIntracomm leaves there) */
  jobject r = (me == root || (flags & MPJX_FLAG_FAITHFUL)) ? recv : NULL;
  if (hb_prepare(env, send, soff, type, count, &hs, err, sizeof err, "Reduce sendbuf"))
    hb_prepare(env, r, roff, type, count, &hr, err, sizeof err, "Reduce recvbuf");
  else
    memset(&hr, 0, sizeof hr);
  hb_pin(env, &hs, 1, 0);
  hb_pin(env, &hr, 0, 1);
  int rc = mpjx_reduce_host(COMM(comm), hs.data, hr.data, count, type, op, root, (unsigned)flags);
  if (err[0] && !rc) rc = MPJX_ERR_ARG; /* cannot happen: libmpjx rejects the NULL buffer */
  hb_close(env, &hr, rc == MPJX_SUCCESS);
  hb_close(env, &hs, 0);
  raise_status(env, rc, err, "Reduce");
}

JNIEXPORT void JNICALL Java_mpi_HipIntracomm_nativeAllreduce(JNIEnv *env, jobject self, jlong comm, jobject send,
                                                             jint soff, jobject recv, jint roff, jint count,
                                                             jint type, jint op, jint flags) {
  (void)self;
  hbuf hs, hr;
  char err[256] = "";
  if (hb_prepare(env, send, soff, type, count, &hs, err, sizeof err, "Allreduce sendbuf"))
    hb_prepare(env, recv, roff, type, count, &hr, err, sizeof err, "Allreduce recvbuf");
  else
    memset(&hr, 0, sizeof hr);
  hb_pin(env, &hs, 1, 0);
  hb_pin(env, &hr, 0, 1);
  int rc = mpjx_allreduce_host(COMM(comm), hs.data, hr.data, count, type, op, (unsigned)flags);
  if (err[0] && !rc) rc = MPJX_ERR_ARG;
  hb_close(env, &hr, rc == MPJX_SUCCESS);
  hb_close(env, &hs, 0);
  raise_status(env, rc, err, "Allreduce");
}

JNIEXPORT void JNICALL Java_mpi_HipIntracomm_nativeReduceScatter(JNIEnv *env, jobject self, jlong comm,
                                                                 jobject send, jint soff, jobject recv, jint roff,
                                                                 jintArray recvcounts, jint type, jint op,
                                                                 jint flags) {
  (void)self;
  int P = 0, me = 0;
  char err[256] = "";
  mpjx_comm_size(COMM(comm), &P);
  mpjx_comm_rank(COMM(comm), &me);
  int64_t *rc64 = (int64_t *)calloc((size_t)(P > 0 ? P : 1), sizeof(int64_t));
  int64_t total = 0;
  if (!recvcounts || (*env)->GetArrayLength(env, recvcounts) < P) {
    snprintf(err, sizeof err, "Reduce_scatter: recvcounts[] shorter than the communicator (%d ranks)", P);
  } else {
    jint *rc32 = (*env)->GetIntArrayElements(env, recvcounts, NULL);
    if (!rc32) {
      snprintf(err, sizeof err, "Reduce_scatter: recvcounts[] not accessible");
    } else {
      for (int i = 0; i < P; i++) {
        rc64[i] = rc32[i];
        total += rc32[i] > 0 ? rc32[i] : 0;
      }
      (*env)->ReleaseIntArrayElements(env, recvcounts, rc32, JNI_ABORT);
    }
  }
  hbuf hs, hr;
  memset(&hs, 0, sizeof hs);
  memset(&hr, 0, sizeof hr);
  if (!err[0] && hb_prepare(env, send, soff, type, total, &hs, err, sizeof err, "Reduce_scatter sendbuf"))
    hb_prepare(env, recv, roff, type, (me >= 0 && me < P) ? rc64[me] : 0, &hr, err, sizeof err,
               "Reduce_scatter recvbuf");
  hb_pin(env, &hs, 1, 0);
  hb_pin(env, &hr, 0, 1);
  /* a recvcounts failure leaves rc64 zeroed: libmpjx then sees NULL buffers with a zero-length call on
   * this rank only; pass NULL counts so it rejects the call (and releases the other ranks) */
  int rc = mpjx_reduce_scatter_host(COMM(comm), hs.data, hr.data, err[0] ? NULL : rc64, type, op, (unsigned)flags);
  if (err[0] && !rc) rc = MPJX_ERR_ARG;
  /* faithful BKT ring (default collectives, typed ops, 2+ ranks): sendbuf was rewritten as the
   * reference rewrites it (PureIntracomm.java:2427-2428), so it is written back too */
  const int send_back = (flags & MPJX_FLAG_FAITHFUL) && !(flags & MPJX_FLAG_OLD_COLLECTIVES) && type < 0x100 && P >= 2;
  hb_close(env, &hr, rc == MPJX_SUCCESS);
  hb_close(env, &hs, rc == MPJX_SUCCESS && send_back);
  free(rc64);
  raise_status(env, rc, err, "Reduce_scatter");
}

JNIEXPORT void JNICALL Java_mpi_HipIntracomm_nativeScan(JNIEnv *env, jobject self, jlong comm, jobject send,
                                                        jint soff, jobject recv, jint roff, jint count, jint type,
                                                        jint op, jint flags) {
  (void)self;
  hbuf hs, hr;
  char err[256] = "";
  if (hb_prepare(env, send, soff, type, count, &hs, err, sizeof err, "Scan sendbuf"))
    hb_prepare(env, recv, roff, type, count, &hr, err, sizeof err, "Scan recvbuf");
  else
    memset(&hr, 0, sizeof hr);
  hb_pin(env, &hs, 1, 0);
  hb_pin(env, &hr, 0, 1);
  int rc = mpjx_scan_host(COMM(comm), hs.data, hr.data, count, type, op, (unsigned)flags);
  if (err[0] && !rc) rc = MPJX_ERR_ARG;
  hb_close(env, &hr, rc == MPJX_SUCCESS);
  hb_close(env, &hs, 0);
  raise_status(env, rc, err, "Scan");
}

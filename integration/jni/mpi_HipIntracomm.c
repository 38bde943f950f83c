/*
 * mpi_HipIntracomm.c — JNI shim between mpi.HipIntracomm (integration/java/mpi/HipIntracomm.java)
 * and libmpjx (include/mpjx.h). New code for a maintainer to build where a JDK exists:
 *
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I<repo>/include \
 *       mpi_HipIntracomm.c -L<repo>/mpjexpress_amd/lib -lmpjx -Wl,-rpath,<repo>/mpjexpress_amd/lib \
 *       -o libmpjx_jni.so
 *
 * It replaces the body of Java_mpjdev_natmpjdev_Intracomm_nativeReduce
 * (src/mpjdev/natmpjdev/lib/mpjdev_natmpjdev_Intracomm.c:410-627): instead of
 * Get<Type>ArrayElements + MPI_Reduce + one JNI upcall per result element, the Java arrays are
 * pinned with GetPrimitiveArrayCritical and handed to the mpjx_*_host entry points as plain
 * pointers (offset applied here, counts widened to int64). Status codes become mpi.MPIException
 * (src/mpi/MPIException.java:42) carrying mpjx_last_error(), where the reference ignored MPI's
 * return code.
 *
 * Not compiled in this repository: the build image has no jni.h.
 */
#include <jni.h>
#include <pthread.h>
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
  (*env)->GetByteArrayRegion(env, uid, 0, (jsize)sizeof id, (jbyte *)&id);
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
  (*env)->GetByteArrayRegion(env, uid, 0, (jsize)sizeof id, (jbyte *)&id);
  int rc = mpjx_comm_init_ipc(&c, size, &id, rank, device);
  if (rc) { throw_mpi(env, rc, "mpjx_comm_init_ipc"); return 0; }
  return (jlong)(intptr_t)c;
}

/* multicore (smpdev): the first rank thread creates every rank's communicator */
static pthread_mutex_t g_smp_mu = PTHREAD_MUTEX_INITIALIZER;
static mpjx_comm_t *g_smp = NULL;
static int g_smp_size = 0;

JNIEXPORT jlong JNICALL Java_mpi_HipIntracomm_nativeInitSmp(JNIEnv *env, jclass cls, jint rank, jint size,
                                                            jint device) {
  (void)cls;
  (void)device;
  pthread_mutex_lock(&g_smp_mu);
  if (!g_smp) {
    int *devs = (int *)calloc((size_t)size, sizeof(int));
    int ndev = 0;
    mpjx_device_count(&ndev);
    for (int r = 0; r < size; r++) devs[r] = ndev > 0 ? r % ndev : 0;
    g_smp = (mpjx_comm_t *)calloc((size_t)size, sizeof(mpjx_comm_t));
    g_smp_size = size;
    int rc = mpjx_comm_init_smp(g_smp, size, devs);
    free(devs);
    if (rc) {
      free(g_smp);
      g_smp = NULL;
      pthread_mutex_unlock(&g_smp_mu);
      throw_mpi(env, rc, "mpjx_comm_init_smp");
      return 0;
    }
  }
  mpjx_comm_t c = (rank >= 0 && rank < g_smp_size) ? g_smp[rank] : NULL;
  pthread_mutex_unlock(&g_smp_mu);
  return (jlong)(intptr_t)c;
}

/* Pin a Java primitive array (or take a direct ByteBuffer's address) and apply the element offset. */
typedef struct {
  jarray arr;
  void *base;
  int critical;
} pinned;

static char *pin(JNIEnv *env, jobject buf, int elem_offset, int type, pinned *p) {
  p->arr = NULL;
  p->base = NULL;
  p->critical = 0;
  if (!buf) return NULL;
  void *addr = (*env)->GetDirectBufferAddress(env, buf);  /* mpjbuf NIOBuffer / direct ByteBuffer */
  if (!addr) {
    p->arr = (jarray)buf;
    addr = (*env)->GetPrimitiveArrayCritical(env, p->arr, NULL);
    p->critical = 1;
  }
  p->base = addr;
  /* offsets are Java array indices, i.e. base elements (half a pair for the *2 types) */
  size_t base = (size_t)mpjx_type_size(type & 0xff);
  return addr ? (char *)addr + (size_t)elem_offset * base : NULL;
}

static void unpin(JNIEnv *env, pinned *p, int write_back) {
  if (p->critical && p->base) (*env)->ReleasePrimitiveArrayCritical(env, p->arr, p->base, write_back ? 0 : JNI_ABORT);
}

#define COMM(c) ((mpjx_comm_t)(intptr_t)(c))

JNIEXPORT void JNICALL Java_mpi_HipIntracomm_nativeReduce(JNIEnv *env, jobject self, jlong comm, jobject send,
                                                          jint soff, jobject recv, jint roff, jint count,
                                                          jint type, jint op, jint root, jint flags) {
  (void)self;
  pinned ps, pr;
  int me = -1;
  mpjx_comm_rank(COMM(comm), &me);
  char *s = pin(env, send, soff, type, &ps);
  char *r = (me == root) ? pin(env, recv, roff, type, &pr) : (pr.critical = 0, (char *)NULL);
  int rc = mpjx_reduce_host(COMM(comm), s, r, count, type, op, root, (unsigned)flags);
  if (me == root) unpin(env, &pr, 1);
  unpin(env, &ps, 0);
  if (rc) throw_mpi(env, rc, "Reduce");
}

JNIEXPORT void JNICALL Java_mpi_HipIntracomm_nativeAllreduce(JNIEnv *env, jobject self, jlong comm, jobject send,
                                                             jint soff, jobject recv, jint roff, jint count,
                                                             jint type, jint op, jint flags) {
  (void)self;
  pinned ps, pr;
  char *s = pin(env, send, soff, type, &ps);
  char *r = pin(env, recv, roff, type, &pr);
  int rc = mpjx_allreduce_host(COMM(comm), s, r, count, type, op, (unsigned)flags);
  unpin(env, &pr, 1);
  unpin(env, &ps, 0);
  if (rc) throw_mpi(env, rc, "Allreduce");
}

JNIEXPORT void JNICALL Java_mpi_HipIntracomm_nativeReduceScatter(JNIEnv *env, jobject self, jlong comm,
                                                                 jobject send, jint soff, jobject recv, jint roff,
                                                                 jintArray recvcounts, jint type, jint op,
                                                                 jint flags) {
  (void)self;
  int P = 0;
  mpjx_comm_size(COMM(comm), &P);
  int64_t *rc64 = (int64_t *)calloc((size_t)P, sizeof(int64_t));
  jint *rc32 = (*env)->GetIntArrayElements(env, recvcounts, NULL);
  for (int i = 0; i < P; i++) rc64[i] = rc32[i];
  (*env)->ReleaseIntArrayElements(env, recvcounts, rc32, JNI_ABORT);
  pinned ps, pr;
  char *s = pin(env, send, soff, type, &ps);
  char *r = pin(env, recv, roff, type, &pr);
  int rc = mpjx_reduce_scatter_host(COMM(comm), s, r, rc64, type, op, (unsigned)flags);
  unpin(env, &pr, 1);
  unpin(env, &ps, 0);
  free(rc64);
  if (rc) throw_mpi(env, rc, "Reduce_scatter");
}

JNIEXPORT void JNICALL Java_mpi_HipIntracomm_nativeScan(JNIEnv *env, jobject self, jlong comm, jobject send,
                                                        jint soff, jobject recv, jint roff, jint count, jint type,
                                                        jint op, jint flags) {
  (void)self;
  pinned ps, pr;
  char *s = pin(env, send, soff, type, &ps);
  char *r = pin(env, recv, roff, type, &pr);
  int rc = mpjx_scan_host(COMM(comm), s, r, count, type, op, (unsigned)flags);
  unpin(env, &pr, 1);
  unpin(env, &ps, 0);
  if (rc) throw_mpi(env, rc, "Scan");
}

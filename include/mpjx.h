/*
 * mpjx.h — C ABI of libmpjx, the MI355X-native (gfx950) reduction-collective path of MPJ Express.
 *
 * Drop-in boundary. The reference routes Reduce/Allreduce/Reduce_scatter/Scan through an
 * IntracommImpl strategy (src/mpi/IntracommImpl.java:426-503, chosen at src/mpi/Intracomm.java:63-67);
 * its only native reduction is the JNI entry point
 *   Java_mpjdev_natmpjdev_Intracomm_nativeReduce(JNIEnv*, jobject, jlong comm, jobject sendArray,
 *       jobject recvDirectBuffer, jint count, jint type, jint op, jint root)
 *   (src/mpjdev/natmpjdev/lib/mpjdev_natmpjdev_Intracomm.c:410-627, bound at
 *    src/mpjdev/natmpjdev/Intracomm.java:723-737)
 * which hands `type.baseType` and `op.opCode` to MPI_Reduce. Every entry point below takes those
 * same integer codes unchanged, plain pointers and 64-bit element counts; nothing here mentions
 * torch, JNI or Java types. INTEGRATION.md shows the JNI shim and the HipIntracomm class a
 * maintainer adds on the Java side.
 *
 * Conventions
 *  - Every function returns an int status: MPJX_SUCCESS (0) or a negative MPJX_ERR_* code;
 *    mpjx_strerror() names it and mpjx_last_error() gives the calling thread's detail message
 *    (the reference throws mpi.MPIException: src/mpi/MPIException.java:42).
 *  - Device-pointer entry points ENQUEUE work on `stream` (a hipStream_t passed as void*; NULL =
 *    the communicator's own stream) and return without waiting; mpjx_comm_synchronize() waits.
 *    Consecutive calls on one communicator are ordered: a call on another stream than the previous
 *    call's waits for that stream, so the previous call's stream must stay valid until then (or
 *    until mpjx_comm_synchronize / mpjx_comm_destroy).
 *  - Element semantics are the reference's typed Op bodies (acc[i] = in[i] (op) acc[i]) with Java
 *    arithmetic: integer wrap-around, char unsigned, MAX/MIN as `if (in > acc) acc = in`
 *    (NaN never replaces, +0/-0 ties keep the accumulator), IEEE float/double with subnormals.
 *  - Combine ORDER follows the reference algorithm selected by `flags`, so float/double results
 *    are bit-identical to the reference's pure-Java collectives on the same inputs.
 *  - Device entry points check that every buffer is GPU-accessible (device, managed, or host memory
 *    allocated with hipHostMalloc) before any kernel runs, and return MPJX_ERR_ARG otherwise.
 *  - A collective call that fails on a rank (rejected arguments, a bad root, a failed step part-way)
 *    marks multicore and IPC worlds failed: the other ranks' matching and later calls return
 *    MPJX_ERR_INTERNAL instead of waiting for it (destroy and re-create the communicator). In RCCL
 *    worlds the other ranks wait, as MPI ranks do (MPJX_RCCL_TIMEOUT_S ends the wait), and at P > 1
 *    the failing rank's communicator is aborted: its later calls return MPJX_ERR_RCCL instead of
 *    pairing with the peers' pending operation.
 *  - The caller owns every buffer; the library owns streams, events and device scratch, cached
 *    per communicator. Calls on one communicator must come from one thread at a time (MPI
 *    semantics); several communicators may be driven concurrently from different threads.
 */
#ifndef MPJX_H
#define MPJX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPJX_VERSION 100 /* 1.0.0 */

/* mpi.Datatype.baseType codes (src/mpi/Datatype.java:57-66); byte sizes src/mpi/BasicType.java:50-140 */
enum {
  MPJX_BYTE = 1,    /* Java byte,    int8  */
  MPJX_CHAR = 2,    /* Java char,    uint16 */
  MPJX_SHORT = 3,   /* Java short,   int16 */
  MPJX_BOOLEAN = 4, /* Java boolean, uint8 0/1 */
  MPJX_INT = 5,     /* Java int,     int32 */
  MPJX_LONG = 6,    /* Java long,    int64 */
  MPJX_FLOAT = 7,   /* Java float,   IEEE binary32 */
  MPJX_DOUBLE = 8   /* Java double,  IEEE binary64 */
};

/* (value, index) pair types MPI.SHORT2/INT2/LONG2/FLOAT2/DOUBLE2 = Datatype.Contiguous(2, base)
 * (src/mpi/MPI.java:110-114): code = 0x100 | base code; one element = one pair; only MAXLOC/MINLOC. */
enum {
  MPJX_SHORT2 = 0x103, MPJX_INT2 = 0x105, MPJX_LONG2 = 0x106, MPJX_FLOAT2 = 0x107, MPJX_DOUBLE2 = 0x108
};

/* mpi.Op.opCode values (src/mpjdev/Constants.java:53-64; MPI.MAX..MPI.MINLOC at src/mpi/MPI.java:117-130) */
enum {
  MPJX_MAX = 1, MPJX_MIN = 2, MPJX_SUM = 3, MPJX_PROD = 4, MPJX_LAND = 5,
  MPJX_BAND = 6, MPJX_LOR = 7, MPJX_BOR = 8, MPJX_LXOR = 9, MPJX_BXOR = 10,
  MPJX_MAXLOC = 11, /* src/mpi/Maxloc.java: larger value wins; equal values keep the smaller index */
  MPJX_MINLOC = 12  /* src/mpi/Minloc.java: smaller value wins; equal values keep the smaller index */
};

/* status codes */
enum {
  MPJX_SUCCESS = 0,
  MPJX_ERR_ARG = -1,         /* bad pointer/count/rank/root argument */
  MPJX_ERR_OP_TYPE = -2,     /* the reference's *Worker.getWorker throws for this (op, type) */
  MPJX_ERR_HIP = -3,         /* HIP runtime error */
  MPJX_ERR_RCCL = -4,        /* RCCL error */
  MPJX_ERR_NO_DEVICE = -5,   /* no usable gfx950 device / kernel image */
  MPJX_ERR_UNSUPPORTED = -6, /* combination not provided by this build */
  MPJX_ERR_INTERNAL = -7
};

/* flags (collectives) */
#define MPJX_FLAG_OLD_COLLECTIVES 0x1u /* mirror conf `mpjexpress.mpi.old.collectives=true`
                                          (MPI.isOldSelected, src/mpi/MPI.java:70,266): flat-tree
                                          orders of FT_Reduce / FT_Allreduce / FT_Reduce_scatter */
#define MPJX_FLAG_FAITHFUL 0x2u        /* reproduce the reference's observable state, defects
                                          included. Results: BOR/BXOR never combine (every perform
                                          keeps the accumulator; src/mpi/BorInt.java:50 overloads
                                          instead of overriding src/mpi/Op.java:56); the P>=3 bucket
                                          Reduce_scatter result (src/mpi/PureIntracomm.java:2377-2439).
                                          Buffers written BEYOND the MPI contract (see each call):
                                          - mpjx_reduce, default order: EVERY rank's recvbuf (count
                                            elements) = the MST reduction of the largest sub-tree the
                                            rank roots (:1937-1939 copy send into recvbuf and reduce
                                            there); the root's is the result;
                                          - mpjx_reduce, with MPJX_FLAG_OLD_COLLECTIVES: every
                                            non-root's recvbuf = a copy of its sendbuf (:2038,2052);
                                          - mpjx_reduce_scatter, default order, P>=2, non-pair types:
                                            the caller's SENDBUF is overwritten (:2427-2428): its own
                                            block (at sum(recvcounts[0..rank))) = the rank's result,
                                            every other element x = x (op) 0 folded P-1 times.
                                          Not reproduced: the nonzero-offset loop-bound quirk (no
                                          offsets cross this ABI) and FT_Reduce_scatter's full-length
                                          recvbuf writes (the Java strategy keeps those calls,
                                          INTEGRATION.md). */

#define MPJX_FLAG_SEND_BIG_ENDIAN 0x4u /* sendbuf elements are big-endian: an mpjbuf section payload as
                                          niodev delivers it (src/mpjbuf/NIOBuffer.java:42, encoding
                                          never changed, src/mpjbuf/Buffer.java:5414) */
#define MPJX_FLAG_RECV_BIG_ENDIAN 0x8u /* write recvbuf big-endian (ready to send on as mpjbuf) */
#define MPJX_FLAG_BLOCKING 0x10u       /* return only once the call's results are complete, as if followed by
                                          mpjx_comm_synchronize (the mpiJava calls are blocking:
                                          src/mpi/Intracomm.java:740-885). In multicore mode the ranks then
                                          end a call with a host rendezvous after the launching rank's
                                          stream has drained, instead of ordering every rank's stream after
                                          it by events. Ignored by the *_host variants (synchronous anyway). */
/* Both byte-order flags are part of the call's datatype: pass the same ones on every rank, like
 * `type` and `op`. The combine kernels swap in registers (no extra pass over the vector). */

typedef struct mpjx_comm *mpjx_comm_t;
typedef struct {
  char internal[128]; /* == ncclUniqueId */
} mpjx_unique_id;

/* ---- library ------------------------------------------------------------------------------- */
int mpjx_version(void);
/* The HIP runtime and RCCL versions this process actually bound (not the headers it was built
 * against: a JVM binds /opt/rocm's, a Python process the ones torch loaded first). Either pointer may
 * be NULL. MPJX_ERR_HIP if the HIP runtime does not answer. */
int mpjx_runtime_versions(int *hip_runtime, int *rccl);
const char *mpjx_strerror(int status);
const char *mpjx_last_error(void); /* detail of the calling thread's last failure */
/* Bytes per element of a datatype code, 0 if unknown (BasicType.byteSize). */
int mpjx_type_size(int type);
/* MPJX_SUCCESS if the reference has a typed worker for (op, type), else MPJX_ERR_OP_TYPE
 * (e.g. SUM on BOOLEAN: src/mpi/SumWorker.java:60; BAND on DOUBLE: src/mpi/BandWorker.java:60). */
int mpjx_op_check(int op, int type);
/* Number of visible devices that this build can run on (gfx950). */
int mpjx_device_count(int *count);

/* ---- element-wise combine (the typed Op.perform loop, src/mpi/SumDouble.java:49-55) --------- */
/* inout[i] = in[i] (op) inout[i], i in [0, count), device pointers. Replaces one
 * createInitialBuffer/perform/getResultant round trip (src/mpi/PureIntracomm.java:1979-1986). */
int mpjx_combine(int op, int type, void *inout, const void *in, int64_t count, void *stream);

/* P-way combine in a reference ORDER: the local reduction step that follows an exchange (the
 * reference performs it edge by edge inside MST_Reduce / FT_Reduce / Scan). `in[0..P)` are P
 * operand slices of `count` elements (index = rank); out[0] receives the result slice, or for
 * MPJX_ORDER_SCAN out[0..P) receive every rank's inclusive prefix. Device pointers; an output may
 * alias an input.
 *   MPJX_ORDER_MST   out[0] = MST_Reduce tree over ranks 0..P-1 rooted at `root` (PureIntracomm.java:1943-1992)
 *   MPJX_ORDER_FOLD  out[0] = in[P-1] (op) (... (op) (in[1] (op) in[0]))  (FT_Reduce with in[0] = x_root)
 *   MPJX_ORDER_SCAN  out[r] = in[r-1] (op) (... (op) (in[0] (op) in[r]))   (Scan, :2526-2544)        */
enum { MPJX_ORDER_FOLD = 0, MPJX_ORDER_MST = 1, MPJX_ORDER_SCAN = 2 };
int mpjx_combine_multi(int op, int type, int order, int P, const void *const *in, void *const *out,
                       int64_t count, int root, unsigned flags, void *stream);

/* mpjbuf section header at byte `pos` (rounded up to the 8-byte ALIGNMENT_UNIT) of a static buffer
 * of `nbytes` (src/mpjbuf/Buffer.java:609-704 putSectionHeader/getSectionHeader: type code byte,
 * big-endian int32 element count at +4, payload at +8 = SECTION_OVERHEAD). Returns the datatype
 * code (mpjbuf.Type code + 1 for the 8 basic types, src/mpjbuf/Type.java:66-73), the element count
 * and the payload's byte position, so a caller can reduce a niodev payload in place with the
 * BIG_ENDIAN flags instead of unpacking it on the host. Host memory only; no device work. */
int mpjx_mpjbuf_section(const void *buf, int64_t nbytes, int64_t pos, int *type, int64_t *count,
                        int64_t *data_pos);

/* The per-edge combine of MST_Reduce on a packed message, with the section walk on the device:
 * acc[i] = payload[i] (op) acc[i] for i < count, where the payload is the big-endian element run of
 * the mpjbuf sections at the start of `msg` (a static-buffer image of msg_bytes bytes, e.g. a niodev
 * message in device memory or in pinned host memory; src/mpjbuf/Buffer.java:609-704 section headers,
 * NIOBuffer.java:520-563 big-endian elements; a message may hold several sections of the type, read
 * in order; pair types are sections of their base type). Replaces the host unpack + perform of
 * PureIntracomm.java:1979-1986 with one HBM pass. The kernel reads the headers: a wrong type code
 * (1), element counts that do not add up to count (2), a header or payload past msg_bytes (3) or more
 * than 64 sections (4) leave acc untouched and store that code into *status (a device-accessible int
 * the caller zeroes); 0 stays there on success. Asynchronous on `stream`. flags: MPJX_FLAG_FAITHFUL
 * only. */
#define MPJX_MPJBUF_BAD_TYPE 1
#define MPJX_MPJBUF_BAD_COUNT 2
#define MPJX_MPJBUF_OVERRUN 3
#define MPJX_MPJBUF_TOO_MANY_SECTIONS 4
int mpjx_mpjbuf_combine(int op, int type, void *acc, const void *msg, int64_t msg_bytes, int64_t count,
                        int *status, unsigned flags, void *stream);

/* ---- communicators ----------------------------------------------------------------------------- */
/* One process per GPU over RCCL (the niodev/native-device deployment): rank 0 creates the id,
 * every rank calls mpjx_comm_init_rank with it. Replaces MPJDev.init + the COMM_WORLD Intracomm
 * (src/mpi/MPI.java:298-305). Blocking waits on such a communicator poll RCCL's asynchronous error
 * state; an error, or a call still incomplete after MPJX_RCCL_TIMEOUT_S seconds (unset: no limit),
 * aborts the communicator (ncclCommAbort) and returns MPJX_ERR_RCCL, and every later call on it fails
 * the same way, instead of the rank hanging on a dead peer. The routing knobs MPJX_RCCL_P2P (grouped
 * send/recv exchanges) and MPJX_RCCL_NATIVE / MPJX_RCCL_NATIVE_P2 (one ncclAllReduce where the result is
 * order-free) are read HERE, once per communicator, and checked equal on every rank (collective; ranks
 * that differ all get MPJX_ERR_ARG); later changes to the environment do not affect the communicator. */
int mpjx_get_unique_id(mpjx_unique_id *id);
int mpjx_comm_init_rank(mpjx_comm_t *comm, int nranks, const mpjx_unique_id *id, int rank, int device);
/* Multicore mode: nranks ranks that are threads of THIS process (smpdev,
 * src/runtime/starter/MulticoreStarter.java:309-322), rank r on devices[r] (devices may repeat).
 * Fills comms[0..nranks). Each rank's thread then drives its own comm. When every device pair has
 * peer access, the collectives read and write the other ranks' buffers directly (one kernel, two
 * host rendezvous; all ranks on one device: rank 0 launches for everyone), so every rank's buffers
 * must stay valid until all ranks' calls have returned and their streams passed the call.
 * MPJX_SMP_COPY=1 selects copy-based exchanges instead. */
int mpjx_comm_init_smp(mpjx_comm_t *comms, int nranks, const int *devices);
/* The same multicore world formed by the rank threads one by one (smpdev: every rank thread runs
 * MPI.Init and creates each communicator itself, MulticoreStarter.java:309-322; NativeIntracomm's
 * Split/Create, src/mpi/NativeIntracomm.java:160-215): every rank thread of a world calls it with
 * the world's id (any 128 bytes unique to it, shared over the host Bcast) and all ranks' devices.
 * The first caller creates every handle; each caller gets its own. Non-blocking. Every caller must
 * pass the same nranks and devices[] (a mismatch is MPJX_ERR_ARG). The registry keeps a world until
 * its last rank has taken its handle: a rank thread that never arrives leaves the others' handles
 * usable only for calls that do not need it (a collective would wait for it). */
int mpjx_comm_init_smp_rank(mpjx_comm_t *comm, int nranks, const mpjx_unique_id *id, int rank,
                            const int *devices);
/* Processes of one node without RCCL (several niodev/native-device ranks on one host, one per GPU or
 * several sharing a GPU): each rank maps the other ranks' device buffers through HIP IPC and every
 * collective runs on the direct engine above (one P-way kernel per rank reading every rank's send
 * block and writing every rank's recv block over xGMI, between two host barriers). `id` is any 128
 * bytes unique to this world, shared out of band (mpjx_get_unique_id works); the ranks rendezvous
 * through a POSIX shared-memory segment named from it, so they must share /dev/shm. Buffers must
 * be hipMalloc'd device memory (any offset into an allocation). A rank that fails or does not
 * arrive within MPJX_IPC_TIMEOUT_S seconds (default 300) makes every rank's call fail instead of
 * hanging. MPJX_SMP_COPY=1 selects copy-based exchanges (pulls from the mapped buffers). */
int mpjx_comm_init_ipc(mpjx_comm_t *comm, int nranks, const mpjx_unique_id *id, int rank, int device);
int mpjx_comm_destroy(mpjx_comm_t comm);
int mpjx_comm_rank(mpjx_comm_t comm, int *rank);
int mpjx_comm_size(mpjx_comm_t comm, int *size);
int mpjx_comm_device(mpjx_comm_t comm, int *device);
int mpjx_comm_stream(mpjx_comm_t comm, void **stream);
int mpjx_comm_synchronize(mpjx_comm_t comm);
int mpjx_barrier(mpjx_comm_t comm);

/* ---- collectives on device-resident buffers (IntracommImpl, src/mpi/IntracommImpl.java:426-503) ---- */
/* Intracomm.Reduce (src/mpi/Intracomm.java:740-760 -> PureIntracomm.java:1923-1992): result on
 * `root`. Default order = MST_Reduce tree. Without MPJX_FLAG_FAITHFUL the recvbuf of other ranks is
 * neither read nor written (may be NULL there). With MPJX_FLAG_FAITHFUL recvbuf is significant and
 * WRITTEN on every rank: its MST sub-tree partial (default), or a copy of its own sendbuf (with
 * MPJX_FLAG_OLD_COLLECTIVES) — see MPJX_FLAG_FAITHFUL. */
int mpjx_reduce(mpjx_comm_t comm, const void *sendbuf, void *recvbuf, int64_t count, int type, int op,
                int root, unsigned flags, void *stream);
/* Intracomm.Allreduce (src/mpi/Intracomm.java:787-793 -> PureIntracomm.java:2168-2185): default
 * order = MST_Reduce(root 0) + MST_Bcast, identical bits on every rank. In-place allowed. */
int mpjx_allreduce(mpjx_comm_t comm, const void *sendbuf, void *recvbuf, int64_t count, int type,
                   int op, unsigned flags, void *stream);
/* Intracomm.Reduce_scatter (src/mpi/Intracomm.java:833-840 -> PureIntracomm.java:2355-2456):
 * rank r receives recvcounts[r] elements (block r of the reduced vector). sendbuf is read only,
 * except with MPJX_FLAG_FAITHFUL (default order, P >= 2, non-pair types), where the call ends by
 * overwriting the caller's sendbuf as the reference's bucket ring does — see MPJX_FLAG_FAITHFUL. */
int mpjx_reduce_scatter(mpjx_comm_t comm, const void *sendbuf, void *recvbuf, const int64_t *recvcounts,
                        int type, int op, unsigned flags, void *stream);
/* Intracomm.Scan (src/mpi/Intracomm.java:879-885 -> PureIntracomm.java:2495-2545): inclusive
 * prefix, rank r gets x_{r-1} (op) (... (op) (x_0 (op) x_r)) — the reference's fold order. */
int mpjx_scan(mpjx_comm_t comm, const void *sendbuf, void *recvbuf, int64_t count, int type, int op,
              unsigned flags, void *stream);
/* Measurement: with enable != 0, mpjx_allreduce, mpjx_reduce_scatter and mpjx_scan record HIP timing
 * events at their phase boundaries on the call's stream (one communicator, cheap, off by default).
 * mpjx_comm_last_phases waits for the last instrumented call and returns its three phase durations in
 * ms and the engine that ran it:
 *   *engine = 1  exchange engine (RCCL, or copy exchanges): exchange #1 / P-way combine / exchange #2
 *                (Reduce_scatter has no exchange #2: ms3[2] ~ 0, or the faithful sendbuf rewrite)
 *   *engine = 2  direct engine (multicore, HIP-IPC): share (incl. IPC pushes + rendezvous) / combine /
 *                fence (incl. IPC copy-out + rendezvous)
 *   *engine = 3  chunk-pipelined Allreduce: ms3[0] = the whole call (its phases overlap), others -1
 *   *engine = 4  one-rank communicator: ms3[1] = the copy send -> recv (ms3[0], ms3[2] ~ 0)
 *   *engine = 5  one-shot (small vectors): all-gather of the whole vectors / combine / - (~0)
 *   *engine = 6  one ncclAllReduce (MPJX_RCCL_NATIVE=1 where the result is order-free): ms3[1]
 * A windowed call (the IPC engine over vectors longer than its staging region) reports its last window.
 * An instrumented call that took a path without phase marks (Reduce, Bcast, ...) makes the next
 * mpjx_comm_last_phases fail with MPJX_ERR_ARG rather than return an earlier call's phases.
 * No reference counterpart (bench.py's N > 1 "phases" breakdown). */
int mpjx_comm_phase_timing(mpjx_comm_t comm, int enable);
int mpjx_comm_last_phases(mpjx_comm_t comm, float *ms3, int *engine);
/* For an instrumented chunk-pipelined Allreduce (*engine = 3): per chunk k, six times in ms from the
 * call's start — exchange #1 start/end (call stream), combine start/end (combine stream), all-gather
 * start/end (gather stream, the transport's second lane) — into ms[6k .. 6k+5], for at most cap / 6
 * chunks; *nchunks = the chunks written. Shows which intervals overlapped. */
int mpjx_comm_pipeline_trace(mpjx_comm_t comm, float *ms, int cap, int *nchunks);
/* Intracomm.Bcast (PureIntracomm.java:592-736), phase 2 of the reference Allreduce. */
int mpjx_bcast(mpjx_comm_t comm, void *buf, int64_t count, int type, int root, void *stream);
/* Intracomm.Gather (PureIntracomm.java:782-1053, MST/FT): `count` elements from every rank land at
 * recvbuf + r*count on the root (recvbuf significant at the root only). */
int mpjx_gather(mpjx_comm_t comm, const void *sendbuf, void *recvbuf, int64_t count, int type, int root,
                void *stream);
/* Intracomm.Scatter (PureIntracomm.java:1055-1171): rank r receives the root's sendbuf + r*count
 * (sendbuf significant at the root only); root delivery step of FT_Reduce_scatter (:2454). */
int mpjx_scatter(mpjx_comm_t comm, const void *sendbuf, void *recvbuf, int64_t count, int type, int root,
                 void *stream);

/* ---- host-resident variants (Java heap arrays / mpjbuf payloads) ---------------------------------
 * Synchronous. Buffers are ordinary host memory; the library stages them through device memory.
 * These are what the JNI shim calls with GetPrimitiveArrayCritical / GetDirectBufferAddress
 * pointers, replacing the body of nativeReduce (mpjdev_natmpjdev_Intracomm.c:455-623).
 * Host-direct form: in multicore mode with every rank on one device, a call of at most one host
 * pipeline chunk (MPJX_HOST_CHUNK_MIB, default 16 MiB) whose buffers on this rank are page-locked at
 * the same address on the device (mpjx_host_alloc, hipHostMalloc) is not staged: the collective's
 * kernel reads and writes those buffers across the host link. Ranks may mix forms. MPJX_HOST_DIRECT=0
 * turns it off. A buffer qualifies only if its whole byte range lies in ONE such allocation (checked
 * against the allocation's start and size); any other range takes the staged form, whose host copies
 * are split at allocation boundaries. MPJX_HOST_ONCE=1: in this form an Allreduce writes its result
 * across the link once, into the first host-direct rank's recvbuf, and the other host-direct ranks copy
 * it host-to-host before the call returns (off by default: slower per call on the measured box). */
int mpjx_reduce_host(mpjx_comm_t comm, const void *sendbuf, void *recvbuf, int64_t count, int type,
                     int op, int root, unsigned flags);
int mpjx_allreduce_host(mpjx_comm_t comm, const void *sendbuf, void *recvbuf, int64_t count, int type,
                        int op, unsigned flags);
int mpjx_reduce_scatter_host(mpjx_comm_t comm, const void *sendbuf, void *recvbuf,
                             const int64_t *recvcounts, int type, int op, unsigned flags);
int mpjx_scan_host(mpjx_comm_t comm, const void *sendbuf, void *recvbuf, int64_t count, int type,
                   int op, unsigned flags);
/* Diagnostic: the form the communicator's last *_host call took on this rank — 1 staged through device
 * buffers (the chunk pipeline), 2 host-direct (the kernel loads and stores the host buffers), 0 none
 * yet. No reference counterpart (tests and latency runs read it). */
int mpjx_comm_last_host_form(mpjx_comm_t comm, int *form);
/* Page-locked host memory the device addresses at the same pointer (hipHostMalloc): staging for a
 * caller whose own arrays cannot stay pinned across a call — the JNI shim's multicore rank threads copy
 * Java arrays through it, so the *_host calls above take their host-direct form. No reference
 * counterpart. mpjx_host_free(NULL) is a no-op. */
int mpjx_host_alloc(void **ptr, int64_t bytes);
int mpjx_host_free(void *ptr);

#ifdef __cplusplus
}
#endif
#endif /* MPJX_H */

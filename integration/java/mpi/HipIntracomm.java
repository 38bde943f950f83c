/*
 * HipIntracomm — the Java side of the MI355X reduction path (new code for a maintainer to add to
 * src/mpi; NOT compiled in this repository: the build image has no JDK).
 *
 * Mirrors how NativeIntracomm plugs into the reference (src/mpi/NativeIntracomm.java:42,1072-1115):
 * it extends PureIntracomm, overrides the four reductions, and falls back to super for everything
 * the GPU path does not cover — non-primitive or derived datatypes (baseType > 8, Size() > 1, except
 * MAXLOC/MINLOC on the pair types SHORT2..DOUBLE2, which the GPU path has) and other user-defined
 * ops (op.worker == null) — and, for speed only, for buffers below -Dmpjx.threshold.bytes where PCIe
 * staging would dominate. Split/Create/clone return HipIntracomm, as NativeIntracomm's do
 * (src/mpi/NativeIntracomm.java:160-215), each with a libmpjx communicator of its own. Selected in
 * the Intracomm constructor (src/mpi/Intracomm.java:63-67); see INTEGRATION.md for the patch.
 *
 * Results do not depend on the size threshold, and every rank of a call takes the same side (see
 * route(): it decides from arguments all ranks pass alike — datatype, op, count, recvcounts, Size()
 * and the conf flags — never from the rank-local offsets, or ranks could split between libmpjx and
 * the Java send/recv of one call and deadlock):
 *  - default: MPI semantics at every size. Calls the pure-Java path computes wrongly go to the GPU
 *    whatever their size: BOR/BXOR (never combined, src/mpi/BorInt.java:50 vs Op.java:56) and every
 *    Reduce_scatter (the BKT ring is wrong on 3+ ranks and overwrites sendbuf on 2+,
 *    PureIntracomm.java:2377-2439; FT_Reduce_scatter writes sum(recvcounts) elements into recvbuf,
 *    :2441-2456). A small call with a nonzero offset that stays on the Java path runs on offset-0
 *    copies of this rank's segments (javaCall()), because the typed classes' loop bound (i < count,
 *    SumDouble.java:52) and MST_Reduce's offset mix-up (:1937-1939) would otherwise skip elements.
 *  - -Dmpjx.faithful=true: the reference's own results and buffer contents at every size. GPU calls
 *    pass MPJX_FLAG_FAITHFUL: BOR/BXOR and the BKT defects, every rank's Reduce recvbuf left as
 *    MST_Reduce/FT_Reduce leave it, and the BKT ring's sendbuf overwrite. The offset quirks exist
 *    only on the Java path, so a faithful call goes to the GPU only if NO rank passed an offset (one
 *    pure-Java Allreduce of a flag agrees on it), and FT_Reduce_scatter (old collectives) stays on
 *    the Java path (its recvbuf writes depend on the Java array's length).
 */
package mpi;

import java.io.File;
import java.nio.file.Files;
import java.nio.file.StandardCopyOption;
import java.security.SecureRandom;

public class HipIntracomm extends PureIntracomm {

  static {
    loadShim();
  }

  /** libmpjx_jni.so -> libmpjx.so. In multicore mode every rank thread loads mpi.jar through a class
   *  loader of its own (src/runtime/starter/MulticoreStarter.java:148-193), and the JVM binds a
   *  native library to one class loader only; the later loaders load a private copy of the shim.
   *  The copies are separate shim instances over ONE libmpjx (resolved by soname), whose process-wide
   *  registry (mpjx_comm_init_smp_rank) is where the rank threads' worlds meet. */
  private static void loadShim() {
    try {
      System.loadLibrary("mpjx_jni");
      return;
    } catch (UnsatisfiedLinkError e) {
      if (e.getMessage() == null || !e.getMessage().contains("another classloader")) throw e;
    }
    String name = System.mapLibraryName("mpjx_jni");
    for (String dir : System.getProperty("java.library.path", "").split(File.pathSeparator)) {
      File lib = new File(dir, name);
      if (!lib.isFile()) continue;
      try {
        File copy = File.createTempFile("mpjx_jni", ".so");
        copy.deleteOnExit();
        Files.copy(lib.toPath(), copy.toPath(), StandardCopyOption.REPLACE_EXISTING);
        System.load(copy.getAbsolutePath());
        return;
      } catch (java.io.IOException io) {
        throw new UnsatisfiedLinkError("mpjx_jni: " + io);
      }
    }
    throw new UnsatisfiedLinkError(name + " not found on java.library.path");
  }

  /* flags of include/mpjx.h */
  static final int FLAG_OLD_COLLECTIVES = 0x1;
  static final int FLAG_FAITHFUL = 0x2;

  /** Bytes below which the pure-Java path stays cheaper than staging through the GPU (speed only:
   *  the results are the same on both sides of it). */
  static int THRESHOLD_BYTES = Integer.getInteger("mpjx.threshold.bytes", 1 << 20);
  /** Reproduce the reference's defective results (A3 BOR/BXOR, A9 BKT ring) instead of MPI's. */
  static final boolean FAITHFUL = Boolean.getBoolean("mpjx.faithful");
  static final boolean MULTICORE = Boolean.getBoolean("mpjx.multicore");

  private long comm;  // mpjx_comm_t of this communicator (0 once freed)

  HipIntracomm(mpjdev.Comm mpjdevComm, mpi.Group group) throws MPIException {
    super(mpjdevComm, group);
    comm = initNative();
  }

  HipIntracomm(mpjdev.Comm mpjdevComm, mpjdev.Group group) throws MPIException {
    super(mpjdevComm, group);
    comm = initNative();
  }

  /** Collective over this communicator's ranks: every rank creates its libmpjx handle. The world id
   *  and (multicore) the ranks' devices travel over the pure-Java Bcast/Allgather of this very
   *  communicator, so every sub-communicator gets a world of its own. */
  private long initNative() throws MPIException {
    int rank = Rank(), size = Size();
    int worldRank = MPI.COMM_WORLD == null ? rank : MPI.COMM_WORLD.Rank();
    int ndev = Math.max(1, nativeDeviceCount());
    int device = Integer.getInteger("mpjx.device", worldRank % ndev);
    if (MULTICORE) {
      // smpdev: ranks are threads of this JVM (each with its own copy of this class); rank 0 draws a
      // random world id, the first rank thread to arrive with it creates every rank's handle
      byte[] id = new byte[128];
      if (rank == 0) new SecureRandom().nextBytes(id);
      super.Bcast(id, 0, 128, MPI.BYTE, 0);
      int[] mine = new int[] {device};
      int[] devices = new int[size];
      super.Allgather(mine, 0, 1, MPI.INT, devices, 0, 1, MPI.INT);
      return nativeInitSmp(id, rank, size, devices);
    }
    // one JVM per GPU: rank 0 makes the world id, the existing host Bcast hands it out; the engine is
    // RCCL's exchange (default) or the HIP-IPC direct engine (-Dmpjx.engine=ipc, JVMs of one node)
    byte[] uid = new byte[128];
    if (rank == 0) nativeUniqueId(uid);
    super.Bcast(uid, 0, 128, MPI.BYTE, 0);
    return "ipc".equals(System.getProperty("mpjx.engine", "rccl"))
        ? nativeInitIpc(rank, size, device, uid)
        : nativeInitRank(rank, size, device, uid);
  }

  /* ---- communicator constructors: sub-communicators stay on the GPU strategy ---- */

  public IntracommImpl Split(int color, int key) {
    PureIntracomm pure = (PureIntracomm) super.Split(color, key);
    if (pure == null || pure.mpjdevComm == null) return pure;  // not a member of any new group
    try {
      return new HipIntracomm(pure.mpjdevComm, pure.group.mpjdevGroup);
    } catch (Exception e) {
      throw new MPIException(e);
    }
  }

  public IntracommImpl Create(Group group) {
    PureIntracomm pure = (PureIntracomm) super.Create(group);
    if (pure == null || pure.mpjdevComm == null) return pure;  // this rank is outside `group`
    try {
      return new HipIntracomm(pure.mpjdevComm, group.mpjdevGroup);
    } catch (Exception e) {
      throw new MPIException(e);
    }
  }

  public Object clone() {
    return this.Create(this.group);
  }

  /** Releases this communicator's libmpjx handle (reached when the facade forwards Free(), see
   *  INTEGRATION.md; otherwise the handle lives until the process exits, like the reference's
   *  no-op Comm.Free, src/mpi/Comm.java:198). */
  public void Free() throws MPIException {
    if (comm != 0) {
      long c = comm;
      comm = 0;
      nativeFree(c);
    }
  }

  /** Typed ops 1..10 on basic types, or MAXLOC/MINLOC (11/12, User_function ops with an opCode,
   *  src/mpi/MPI.java:127-130) on the pair types SHORT2..DOUBLE2 (Contiguous(2, base)). */
  private static boolean gpuType(Datatype t, Op op) {
    boolean typed = t.baseType >= 1 && t.baseType <= 8 && t.Size() == 1 && op.worker != null
        && op.opCode >= 1 && op.opCode <= 10;
    boolean loc = (op.opCode == 11 || op.opCode == 12) && t.Size() == 2
        && (t.baseType == 3 || (t.baseType >= 5 && t.baseType <= 8));
    return typed || loc;
  }

  /** true: run the call on the GPU; false: PureIntracomm (super). See the class comment. Every
   *  input is the same on every rank (the offsets enter only through agreeNoOffsets, which is itself
   *  collective), so all ranks of a call take the same path. */
  private boolean route(Datatype t, Op op, long count, boolean reduceScatter, int soff, int roff) {
    if (comm == 0 || !gpuType(t, op)) return false;
    boolean big = count * t.Size() * t.byteSize >= THRESHOLD_BYTES;
    if (FAITHFUL) {
      // FT_Reduce_scatter, and the BKT ring's User_function branch on the pair types (it copies
      // recvcounts[me] BASE elements back, half of the pairs, PureIntracomm.java:2421-2425): their
      // buffer contents are not rebuilt on the GPU
      if (reduceScatter && (MPI.isOldSelected || t.Size() == 2)) return false;
      return big && agreeNoOffsets(soff, roff);
    }
    if (op.opCode == 8 || op.opCode == 10) return true;                      // BOR, BXOR (A3)
    if (reduceScatter) return true;                                          // BKT ring (A9), FT recvbuf
    return big;
  }

  /** Collective: true iff every rank's sendoffset and recvoffset are 0 (a pure-Java Allreduce of one
   *  int with MAX, PureIntracomm's own path). Only faithful calls pay it. */
  private boolean agreeNoOffsets(int soff, int roff) {
    int[] mine = {(soff != 0 || roff != 0) ? 1 : 0}, any = new int[1];
    super.Allreduce(mine, 0, any, 0, 1, MPI.INT, MPI.MAX);
    return any[0] == 0;
  }

  /** A new array of buf's component type holding buf[off, off + len) (copyIn) or zeros. */
  private static Object segment(Object buf, int off, int len, boolean copyIn) {
    Object w = java.lang.reflect.Array.newInstance(buf.getClass().getComponentType(), Math.max(len, 0));
    if (copyIn && len > 0) System.arraycopy(buf, off, w, 0, len);
    return w;
  }

  /** Default mode, a call staying on the Java path: with nonzero offsets, run super on offset-0
   *  segments of this rank's buffers (MPI semantics; a rank-local decision that needs no agreement,
   *  the message pattern is the same either way) and copy the result back where it is significant. */
  private interface JavaColl { void run(Object s, int so, Object r, int ro) throws MPIException; }

  private void javaCall(Object sendbuf, int soff, int sendLen, Object recvbuf, int roff, int recvLen,
      boolean recvSignificant, JavaColl coll) throws MPIException {
    if (FAITHFUL || (soff == 0 && roff == 0)) {
      coll.run(sendbuf, soff, recvbuf, roff);
      return;
    }
    Object s = segment(sendbuf, soff, sendLen, true);
    Object r = segment(recvbuf != null ? recvbuf : sendbuf, roff, recvLen, false);
    coll.run(s, 0, r, 0);
    if (recvSignificant && recvbuf != null && recvLen > 0) System.arraycopy(r, 0, recvbuf, roff, recvLen);
  }

  /** C-ABI type code (include/mpjx.h): baseType, or 0x100 | baseType for the pair types. */
  private static int code(Datatype t) {
    return t.Size() == 2 ? (0x100 | t.baseType) : t.baseType;
  }

  private int flags() {
    return (MPI.isOldSelected ? FLAG_OLD_COLLECTIVES : 0) | (FAITHFUL ? FLAG_FAITHFUL : 0);
  }

  public void Reduce(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset, final int count,
      final Datatype datatype, final Op op, final int root) throws MPIException {
    if (!route(datatype, op, count, false, sendoffset, recvoffset)) {
      int len = count * datatype.size;
      javaCall(sendbuf, sendoffset, len, recvbuf, recvoffset, len, Rank() == root, new JavaColl() {
        public void run(Object s, int so, Object r, int ro) throws MPIException {
          HipIntracomm.super.Reduce(s, so, r, ro, count, datatype, op, root);
        }
      });
      return;
    }
    nativeReduce(comm, sendbuf, sendoffset, recvbuf, recvoffset, count, code(datatype),
        op.opCode, root, flags());
  }

  public void Allreduce(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset, final int count,
      final Datatype datatype, final Op op) throws MPIException {
    if (!route(datatype, op, count, false, sendoffset, recvoffset)) {
      int len = count * datatype.size;
      javaCall(sendbuf, sendoffset, len, recvbuf, recvoffset, len, true, new JavaColl() {
        public void run(Object s, int so, Object r, int ro) throws MPIException {
          HipIntracomm.super.Allreduce(s, so, r, ro, count, datatype, op);
        }
      });
      return;
    }
    nativeAllreduce(comm, sendbuf, sendoffset, recvbuf, recvoffset, count, code(datatype),
        op.opCode, flags());
  }

  public void Reduce_scatter(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset,
      int[] recvcounts, Datatype datatype, Op op) throws MPIException {
    long total = 0;
    for (int i = 0; i < Size(); i++) total += recvcounts[i];
    if (!route(datatype, op, total, true, sendoffset, recvoffset)) {
      // faithful only (default mode sends every Reduce_scatter to the GPU): the reference's own call
      super.Reduce_scatter(sendbuf, sendoffset, recvbuf, recvoffset, recvcounts, datatype, op);
      return;
    }
    nativeReduceScatter(comm, sendbuf, sendoffset, recvbuf, recvoffset, recvcounts,
        code(datatype), op.opCode, flags());
  }

  public void Scan(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset, final int count,
      final Datatype datatype, final Op op) throws MPIException {
    if (!route(datatype, op, count, false, sendoffset, recvoffset)) {
      int len = count * datatype.size;
      javaCall(sendbuf, sendoffset, len, recvbuf, recvoffset, len, true, new JavaColl() {
        public void run(Object s, int so, Object r, int ro) throws MPIException {
          HipIntracomm.super.Scan(s, so, r, ro, count, datatype, op);
        }
      });
      return;
    }
    nativeScan(comm, sendbuf, sendoffset, recvbuf, recvoffset, count, code(datatype),
        op.opCode, flags());
  }

  /* ---- JNI (integration/jni/mpi_HipIntracomm.c); failures throw mpi.MPIException ---- */
  private static native int nativeDeviceCount();
  private static native void nativeUniqueId(byte[] uid);
  private static native long nativeInitRank(int rank, int size, int device, byte[] uid);
  private static native long nativeInitSmp(byte[] id, int rank, int size, int[] devices);
  private static native void nativeFree(long comm);
  private static native long nativeInitIpc(int rank, int size, int device, byte[] uid);
  private native void nativeReduce(long comm, Object send, int soff, Object recv, int roff,
      int count, int type, int op, int root, int flags);
  private native void nativeAllreduce(long comm, Object send, int soff, Object recv, int roff,
      int count, int type, int op, int flags);
  private native void nativeReduceScatter(long comm, Object send, int soff, Object recv, int roff,
      int[] recvcounts, int type, int op, int flags);
  private native void nativeScan(long comm, Object send, int soff, Object recv, int roff,
      int count, int type, int op, int flags);
}

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
 * Results do not depend on the size threshold (see route()):
 *  - default: MPI semantics at every size. Calls the pure-Java path computes wrongly go to the GPU
 *    whatever their size: BOR/BXOR (never combined, src/mpi/BorInt.java:50 vs Op.java:56),
 *    Reduce_scatter on 3+ ranks (BKT ring, PureIntracomm.java:2377-2439) or on pair types, and any
 *    call with a nonzero offset (loop bound i < count, SumDouble.java:52; send/recv offset mix-up,
 *    PureIntracomm.java:1937-1939).
 *  - -Dmpjx.faithful=true: the reference's own results at every size. GPU calls pass
 *    MPJX_FLAG_FAITHFUL (the BOR/BXOR and BKT defects reproduced on the device); calls with a
 *    nonzero offset stay on the Java path at every size, since only it has that loop-bound quirk.
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

  /** true: run the call on the GPU; false: PureIntracomm (super). See the class comment. */
  private boolean route(Datatype t, Op op, long count, int soff, int roff, boolean reduceScatter) {
    if (comm == 0 || !gpuType(t, op)) return false;
    boolean offsets = soff != 0 || roff != 0;
    boolean big = count * t.Size() * t.byteSize >= THRESHOLD_BYTES;
    if (FAITHFUL) return !offsets && big;
    if (op.opCode == 8 || op.opCode == 10) return true;                      // BOR, BXOR (A3)
    if (reduceScatter && (Size() >= 3 || t.Size() == 2)) return true;        // BKT ring (A9), pairs
    if (offsets) return true;                                                // loop bound (A4)
    return big;
  }

  /** C-ABI type code (include/mpjx.h): baseType, or 0x100 | baseType for the pair types. */
  private static int code(Datatype t) {
    return t.Size() == 2 ? (0x100 | t.baseType) : t.baseType;
  }

  private int flags() {
    return (MPI.isOldSelected ? FLAG_OLD_COLLECTIVES : 0) | (FAITHFUL ? FLAG_FAITHFUL : 0);
  }

  public void Reduce(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset, int count,
      Datatype datatype, Op op, int root) throws MPIException {
    if (!route(datatype, op, count, sendoffset, recvoffset, false)) {
      super.Reduce(sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op, root);
      return;
    }
    nativeReduce(comm, sendbuf, sendoffset, recvbuf, recvoffset, count, code(datatype),
        op.opCode, root, flags());
  }

  public void Allreduce(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset, int count,
      Datatype datatype, Op op) throws MPIException {
    if (!route(datatype, op, count, sendoffset, recvoffset, false)) {
      super.Allreduce(sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op);
      return;
    }
    nativeAllreduce(comm, sendbuf, sendoffset, recvbuf, recvoffset, count, code(datatype),
        op.opCode, flags());
  }

  public void Reduce_scatter(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset,
      int[] recvcounts, Datatype datatype, Op op) throws MPIException {
    long total = 0;
    for (int i = 0; i < Size(); i++) total += recvcounts[i];
    if (!route(datatype, op, total, sendoffset, recvoffset, true)) {
      super.Reduce_scatter(sendbuf, sendoffset, recvbuf, recvoffset, recvcounts, datatype, op);
      return;
    }
    nativeReduceScatter(comm, sendbuf, sendoffset, recvbuf, recvoffset, recvcounts,
        code(datatype), op.opCode, flags());
  }

  public void Scan(Object sendbuf, int sendoffset, Object recvbuf, int recvoffset, int count,
      Datatype datatype, Op op) throws MPIException {
    if (!route(datatype, op, count, sendoffset, recvoffset, false)) {
      super.Scan(sendbuf, sendoffset, recvbuf, recvoffset, count, datatype, op);
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

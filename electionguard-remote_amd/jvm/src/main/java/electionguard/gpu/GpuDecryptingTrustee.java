package electionguard.gpu;

import electionguard.core.ElGamalCiphertext;
import electionguard.core.ElementModP;
import electionguard.core.ElementModQ;
import electionguard.core.GenericChaumPedersenProof;
import electionguard.core.GroupContext;
import electionguard.decrypt.CompensatedDecryptionAndProof;
import electionguard.decrypt.DecryptingTrusteeIF;
import electionguard.decrypt.DirectDecryptionAndProof;

import javax.annotation.Nullable;
import java.math.BigInteger;
import java.security.MessageDigest;
import java.security.NoSuchAlgorithmException;
import java.security.SecureRandom;
import java.util.ArrayList;
import java.util.List;
import java.util.Map;

/**
 * DecryptingTrusteeIF on one MI355X: the delegate RunRemoteDecryptingTrustee wraps
 * (src/main/java/electionguard/decrypt/RunRemoteDecryptingTrustee.java:169-193,227-232), with
 * the interface contract of RemoteDecryptingTrusteeProxy.java:30-122:
 *   - one call = one batch = ONE eg_trustee_decrypt_batch (the whole tally of the RPC);
 *   - results in text order;
 *   - failures throw; the gRPC handler turns them into the response's error string
 *     (RunRemoteDecryptingTrustee.java:200-204), which the proxy maps to an empty list.
 *
 * directDecrypt: M_i = pad_i^s, proof (c, v): a = g^u, b = pad^u, c = H(qbar, pad, data, a, b, M),
 * v = u - c s.  compensatedDecrypt: the same with s = P_l(x_i) (the opened key-ceremony backup of
 * missing guardian l) and the recovery key g^{P_l(x_i)} = prod_j K_{l,j}^{x_i^j}.
 * Each trustee process binds its own GPU (device ordinal of its GpuGroupContext).
 */
public final class GpuDecryptingTrustee implements DecryptingTrusteeIF {
  private final GpuGroupContext gpu;
  private final String id;
  private final int xCoordinate;
  private final ElementModP publicKey;
  private final byte[] secret;                                   // s_i, 32 B big-endian
  private final Map<String, ElementModQ> compensatingShares;     // missing guardian l -> P_l(x_i)
  private final Map<String, List<ElementModP>> commitments;      // guardian -> K_{l,0..quorum-1}
  private final SecureRandom random = new SecureRandom();

  public GpuDecryptingTrustee(GpuGroupContext gpu, String id, int xCoordinate, ElementModQ secretKey,
                              ElementModP publicKey, Map<String, ElementModQ> compensatingShares,
                              Map<String, List<ElementModP>> commitments) {
    this.gpu = gpu;
    this.id = id;
    this.xCoordinate = xCoordinate;
    this.publicKey = publicKey;
    this.secret = new byte[EgHip.Q_BYTES];
    GpuGroupContext.put(this.secret, 0, secretKey.byteArray(), EgHip.Q_BYTES);
    this.compensatingShares = Map.copyOf(compensatingShares);
    this.commitments = Map.copyOf(commitments);
  }

  @Override public String id() { return id; }
  @Override public int xCoordinate() { return xCoordinate; }
  @Override public ElementModP electionPublicKey() { return publicKey; }

  @Override
  public List<DirectDecryptionAndProof> directDecrypt(GroupContext group, List<ElGamalCiphertext> texts,
                                                      ElementModQ extendedBaseHash, @Nullable ElementModQ nonce) {
    final int n = texts.size();
    byte[][] r = decryptBatch(secret, texts, extendedBaseHash, nonce);
    List<DirectDecryptionAndProof> out = new ArrayList<>(n);
    for (int i = 0; i < n; i++)
      out.add(new DirectDecryptionAndProof(gpu.elementP(r[0], i), proof(r[1], i)));
    return out;
  }

  @Override
  public List<CompensatedDecryptionAndProof> compensatedDecrypt(GroupContext group, String missingGuardianId,
                                                                List<ElGamalCiphertext> texts,
                                                                ElementModQ extendedBaseHash,
                                                                @Nullable ElementModQ nonce) {
    ElementModQ share = compensatingShares.get(missingGuardianId);
    List<ElementModP> comm = commitments.get(missingGuardianId);
    if (share == null || comm == null)
      throw new IllegalArgumentException("no key-ceremony share from guardian " + missingGuardianId);
    byte[] s = new byte[EgHip.Q_BYTES];
    GpuGroupContext.put(s, 0, share.byteArray(), EgHip.Q_BYTES);
    final int n = texts.size();
    byte[][] r = decryptBatch(s, texts, extendedBaseHash, nonce);
    java.util.Arrays.fill(s, (byte) 0);
    ElementModP recovery = recoveryPublicKey(comm);
    List<CompensatedDecryptionAndProof> out = new ArrayList<>(n);
    for (int i = 0; i < n; i++)
      out.add(new CompensatedDecryptionAndProof(gpu.elementP(r[0], i), proof(r[1], i), recovery));
    return out;
  }

  /** g^{P_l(x_i)} = prod_j K_{l,j}^{x_i^j}: one powP batch + one product on the GPU. */
  private ElementModP recoveryPublicKey(List<ElementModP> comm) {
    final BigInteger q = new BigInteger(EgConstants.Q_HEX, 16), x = BigInteger.valueOf(xCoordinate);
    List<ElementModQ> exps = new ArrayList<>(comm.size());
    BigInteger xj = BigInteger.ONE;
    for (int j = 0; j < comm.size(); j++) {
      exps.add(gpu.elementQ(GpuGroupContext.hex(xj.toString(16), EgHip.Q_BYTES), 0));
      xj = xj.multiply(x).mod(q);
    }
    return gpu.prodP(gpu.powP(comm, exps));
  }

  private GenericChaumPedersenProof proof(byte[] pr, int i) {
    return new GenericChaumPedersenProof(gpu.elementQ(pr, i * 64), gpu.elementQ(pr, i * 64 + 32));
  }

  /** -> {M (n x 512 B), proofs (n x (c, v) 64 B)} from one eg_trustee_decrypt_batch call. */
  private byte[][] decryptBatch(byte[] s, List<ElGamalCiphertext> texts, ElementModQ qbar, @Nullable ElementModQ nonce) {
    final int n = texts.size();
    byte[] qb = new byte[EgHip.Q_BYTES];
    GpuGroupContext.put(qb, 0, qbar.byteArray(), EgHip.Q_BYTES);
    byte[] M = new byte[n * EgHip.P_BYTES], pr = new byte[n * 64];
    EgHip.trusteeDecryptBatch(gpu.handle(), s, qb, GpuGroupContext.packTexts(texts), proofNonces(n, nonce), n, M, pr);
    return new byte[][] {M, pr};
  }

  /**
   * Proof nonces u_i in [1, q): random (the reference passes nonce = null,
   * RunRemoteDecryptingTrustee.java:193,232), or derived as SHA-256(nonce || i) mod q when a
   * nonce is given (deterministic proofs for tests).
   */
  private byte[] proofNonces(int n, @Nullable ElementModQ nonce) {
    final BigInteger q = new BigInteger(EgConstants.Q_HEX, 16);
    byte[] out = new byte[n * EgHip.Q_BYTES];
    for (int i = 0; i < n; i++) {
      BigInteger u;
      do {
        byte[] b = new byte[EgHip.Q_BYTES];
        if (nonce == null) {
          random.nextBytes(b);
        } else {
          try {
            MessageDigest md = MessageDigest.getInstance("SHA-256");
            md.update(nonce.byteArray());
            md.update(BigInteger.valueOf(i).toByteArray());
            b = md.digest();
          } catch (NoSuchAlgorithmException e) {
            throw new IllegalStateException(e);
          }
        }
        u = new BigInteger(1, b).mod(q);
      } while (u.signum() == 0);
      GpuGroupContext.put(out, i * EgHip.Q_BYTES, u.toByteArray(), EgHip.Q_BYTES);
    }
    return out;
  }
}

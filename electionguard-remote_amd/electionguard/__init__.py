"""MI355X-native ElectionGuard group-operation path (drop-in for the batched 4096-bit
modexp path of JohnLCaron/electionguard-remote).  See DESIGN.md and INTEGRATION.md.

Layout mirrors the upstream packages the reference calls into:
  electionguard.core      GroupContext / ElementModP / ElementModQ (KUtils.java:10-12)
  electionguard.ballot    batchEncryption, Verifier, runAccumulateBallots
  electionguard.decrypt   DecryptingTrustee(IF), Decryption
  electionguard.keyceremony  synthetic key ceremony (inputs to the hot path)
  electionguard.util      ConvertCommonProto analog (wire bytes <-> elements)
"""

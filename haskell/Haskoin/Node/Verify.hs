{-# LANGUAGE DuplicateRecordFields #-}
{-# LANGUAGE FlexibleContexts #-}
{-# LANGUAGE OverloadedRecordDot #-}
{-# LANGUAGE OverloadedStrings #-}
{-# LANGUAGE TemplateHaskell #-}

-- | Batch signature verification on MI355X GPUs for a haskoin-node based
-- validator: the drop-in for per-input 'verifyHashSig' (haskoin-core-1.1.0,
-- /root/reference/stack.yaml:10) and 'verifyStdInput'.
--
-- UNCOMPILED in this repository's image (GHC, stack and cabal are absent;
-- SURVEY.md §8(c)). It is written against include/hkv.h and the reference's
-- own idioms, and its byte layout is the one haskoin-node_amd/hkv/records.py
-- (ctypes) implements and tests/test_host.py checks:
--
--   * config record in the style of NodeConfig (src/Haskoin/Node.hs:74-96);
--   * an actor in the style of withChain (src/Haskoin/Node/Chain.hs:277-307):
--     a mailbox and a receive loop under withAsync + link, which coalesces
--     mempool txs into batched GPU calls and never lets a verify failure
--     reach link (re-submit, then haskoin-core's CPU verifyStdInput);
--   * fed by the node's events: blocks and txs arrive as
--     PeerEvent (PeerMessage p (MBlock b)) / (MTx t), which
--     Haskoin.Node.peerEvents (src/Haskoin/Node.hs:151-174) drops into its
--     @_ -> return ()@ arm (:172) and republishes (:174); the application
--     forwards them here with 'verifyBlock' / 'verifyTx'.
--
-- Assumed dependency names (not checkable here): haskoin-core
-- 'exportCompactSig' / 'exportPubKey' / 'txHash' / 'runPutS . serialize',
-- secp256k1-haskell's 'CompactSig' bytes via 'getCompactSig'.
module Haskoin.Node.Verify
  ( VerifierConfig (..),
    Verifier,
    VerifierException (..),
    withVerifier,
    verifyRawBatch,
    verifyHashSigBatch,
    verifyStdInputBatch,
    VerifyConfig (..),
    VerifyEvent (..),
    VerifyActor,
    withVerifyActor,
    verifyBlock,
    verifyTx,
    verifyWithPolicy,
  )
where

import Control.Monad (forM_, when)
import Control.Monad.Logger (MonadLoggerIO, logDebugS, logWarnS)
import Data.Array (listArray, (!))
import Crypto.Secp256k1 (getCompactSig)
import Data.Bits (shiftR, testBit, (.&.))
import Data.ByteString (ByteString)
import qualified Data.ByteString as B
import qualified Data.ByteString.Unsafe as BU
import qualified Data.Text as T
import Data.Word (Word32, Word64, Word8)
import Foreign.C.String (peekCString)
import GHC.Clock (getMonotonicTimeNSec)
import Foreign.Marshal.Alloc (alloca)
import Foreign.Marshal.Array (allocaArray, withArray)
import Foreign.Marshal.Utils (copyBytes, fillBytes, with)
import Foreign.Ptr (Ptr, castPtr, plusPtr)
import Foreign.Storable (peek, peekElemOff, pokeByteOff)
import Haskoin
  ( Block (..),
    BlockHash,
    Ctx,
    Hash256,
    Network,
    PubKey,
    ScriptOutput,
    Sig,
    Tx (..),
    TxHash,
    encodeOutputBS,
    exportCompactSig,
    exportPubKey,
    getSigHashForkId,
    headerHash,
    runPutS,
    serialize,
    txHash,
    verifyStdInput,
  )
import Haskoin.Node.Verify.FFI
import NQE (Mailbox, Publisher, newMailbox, publish, receive, send)
import UnliftIO
  ( Exception,
    MVar,
    MonadIO,
    MonadUnliftIO,
    bracket,
    link,
    liftIO,
    newMVar,
    throwIO,
    timeout,
    try,
    withAsync,
    withMVar,
  )

-- | Configuration, in the style of NodeConfig (Node.hs:74-96).
data VerifierConfig = VerifierConfig
  { -- | GPUs to shard every batch over (0: all visible)
    gpus :: !Int,
    -- | records per GPU call (the pinned host buffer's capacity)
    maxBatch :: !Int
  }

data Verifier = Verifier
  { ctx :: !(Ptr HkvCtx),
    batch :: !(Ptr HkvBatch),
    capacity :: !Int,
    -- | one call at a time uses the pinned buffer
    lock :: !(MVar ())
  }

-- | A device or argument error (a verdict is never an error).
data VerifierException = VerifierException !String !Int
  deriving (Show)

instance Exception VerifierException

check :: String -> Int -> IO ()
check what rc = when (rc /= 0) $ do
  msg <- peekCString =<< c_hkv_strerror (fromIntegral rc)
  throwIO (VerifierException (what <> ": " <> msg) rc)

-- | Open the GPUs, build the fixed-base tables, run the self-check; close on
-- exit (secp256k1-haskell's createContext / withContext, batch-sized).
withVerifier :: (MonadUnliftIO m) => VerifierConfig -> (Verifier -> m a) -> m a
withVerifier cfg = bracket open close
  where
    open = liftIO $ do
      c <- alloca $ \pc -> do
        c_hkv_open (fromIntegral cfg.gpus) 0 pc >>= check "hkv_open" . fromIntegral
        peek pc
      b <- alloca $ \pb -> do
        c_hkv_batch_alloc c (fromIntegral cfg.maxBatch) pb >>= check "hkv_batch_alloc" . fromIntegral
        peek pb
      l <- newMVar ()
      return Verifier {ctx = c, batch = b, capacity = cfg.maxBatch, lock = l}
    close v = liftIO $ do
      c_hkv_batch_free v.batch
      c_hkv_close v.ctx

-- | Write one 168-byte record at @p@ (include/hkv.h):
--   [0,32) msg32 | [32,64) r | [64,96) s | [96] pubkey length |
--   [97,162) pubkey, zero padded | [162,168) zero.
-- Malformed tuples are written as they are: the GPU rejects them exactly
-- as secp256k1_ec_pubkey_parse / parse_compact would (a verdict, not an error).
pokeRecord :: Ptr Word8 -> (ByteString, ByteString, ByteString) -> IO ()
pokeRecord p (msg, sig, pub) = do
  fillBytes p 0 hkvRecordSize
  copyPrefix p 0 32 msg
  copyPrefix p 32 64 sig
  let pl = min 255 (B.length pub)
  pokeByteOff p 96 (fromIntegral pl :: Word8)
  copyPrefix p 97 65 pub
  where
    copyPrefix dst off n bs =
      BU.unsafeUseAsCStringLen bs $ \(src, len) ->
        copyBytes (dst `plusPtr` off) (castPtr src) (min n len)

-- | Bit i of word i/32 is verdict i. O(n): one peekElemOff per verdict
-- straight from the verdict buffer (no list indexing).
readBits :: Int -> Ptr Word32 -> IO [Bool]
readBits n p = mapM bit [0 .. n - 1]
  where
    bit i = (`testBit` (i .&. 31)) <$> peekElemOff p (i `shiftR` 5)

-- | Raw (msg32, compact r||s, SEC1 pubkey bytes) tuples; mode 'hkvLibsecp'
-- is secp256k1_ecdsa_verify, 'hkvHaskoin' is verifyHashSig. Batches larger
-- than the buffer are split; each chunk is one blocking GPU call.
verifyRawBatch :: Verifier -> Word32 -> [(ByteString, ByteString, ByteString)] -> IO [Bool]
verifyRawBatch v mode = fmap concat . mapM one . chunks v.capacity
  where
    one xs = withMVar v.lock $ \_ -> do
      let n = length xs
          nw = (n + 31) `div` 32
      recs <- c_hkv_batch_records v.batch
      forM_ (zip [0 ..] xs) $ \(i, t) -> pokeRecord (recs `plusPtr` (i * hkvRecordSize)) t
      allocaArray nw $ \bits -> do
        c_hkv_verify v.ctx v.batch (fromIntegral n) mode bits >>= check "hkv_verify" . fromIntegral
        readBits n bits

chunks :: Int -> [a] -> [[a]]
chunks _ [] = []
chunks k xs = let (a, b) = splitAt k xs in a : chunks k b

-- | Element i equals @verifyHashSig ctx h_i s_i p_i@ (haskoin-core).
verifyHashSigBatch :: Ctx -> Verifier -> [(Hash256, Sig, PubKey)] -> IO [Bool]
verifyHashSigBatch c v xs =
  verifyRawBatch v hkvHaskoin
    [(runPutS (serialize h), getCompactSig (exportCompactSig c s), exportPubKey c True p) | (h, s, p) <- xs]

-- | Element i equals @verifyStdInput net ctx tx_i input_i so_i value_i@ for
-- P2PK / P2PKH / P2WPKH / multisig prevouts, bare or behind P2SH / P2WSH /
-- P2SH-P2WSH: template match, strict DER + low S (decodeTxSig), the HASH160
-- / SHA-256 script checks, txSigHash / txSigHashForkId, verifyHashSig and
-- the countMulSig walk all run on the GPU from the serialised txs.
verifyStdInputBatch :: Verifier -> Network -> [Tx] -> [(Int, Int, ScriptOutput, Word64)] -> IO [Bool]
verifyStdInputBatch v net txs ins = withMVar v.lock $ \_ -> do
  let raws = map (runPutS . serialize) txs
      offs = scanl (+) 0 (map (fromIntegral . B.length) raws) :: [Word32]
      scripts = map (\(_, _, so, _) -> encodeOutputBS so) ins
      soffs = scanl (+) 0 (map (fromIntegral . B.length) scripts) :: [Word32]
      jobs =
        [ InputJob (fromIntegral t) (fromIntegral i) so (fromIntegral (B.length s)) val
          | ((t, i, _, val), s, so) <- zip3 ins scripts soffs
        ]
      forkid = maybe hkvNoForkId fromIntegral (getSigHashForkId net)
      n = length ins
      nw = (n + 31) `div` 32
  BU.unsafeUseAsCString (B.concat raws) $ \pbytes ->
    BU.unsafeUseAsCString (B.concat scripts) $ \pscripts ->
      withArray offs $ \poffs ->
        withArray jobs $ \pjobs ->
          with (HkvTxs (castPtr pbytes) poffs (fromIntegral (length txs)) (castPtr pscripts) (last soffs)) $ \ptxs ->
            allocaArray nw $ \bits -> do
              c_hkv_verify_std_inputs v.ctx ptxs pjobs (fromIntegral n) forkid bits
                >>= check "hkv_verify_std_inputs" . fromIntegral
              readBits n bits

-- ---------------------------------------------------------------------------
-- The Verify actor (withChain idiom, Chain.hs:277-307)
--
-- Mirrored, policy for policy, by haskoin-node_amd/hkv/actor.py (VerifyActor),
-- which tests/test_gpu_actor.py runs on the GPU.

-- | Where the prevouts come from: the node keeps no UTXO set (headers only,
-- Chain.hs:209-231), so the application supplies (tx index, input index,
-- prevout script, amount) for every input it wants checked.
data VerifyConfig = VerifyConfig
  { net :: !Network,
    -- | secp256k1-haskell context for the CPU re-verify of a failed batch
    secp :: !Ctx,
    verifier :: !Verifier,
    prevouts :: !(Block -> IO [(Int, Int, ScriptOutput, Word64)]),
    txPrevouts :: !(Tx -> IO [(Int, ScriptOutput, Word64)]),
    -- | mempool txs are coalesced into one GPU call of at most this many
    -- inputs (16,384: the pair kernel's range, DESIGN.md §4.2)...
    maxInputs :: !Int,
    -- | ...or of what arrived within this many microseconds of the first
    maxWaitMicros :: !Int,
    -- | GPU re-submissions of a batch whose call failed before the CPU path
    retries :: !Int,
    -- | verdicts are published here
    pub :: !(Publisher VerifyEvent)
  }

data VerifyEvent
  = BlockVerified !BlockHash
  | BlockRejected !BlockHash ![(Int, Int)]
  | TxVerified !TxHash
  | TxRejected !TxHash ![Int]

data VerifyMessage
  = VerifyBlock !Block
  | VerifyTx !Tx

newtype VerifyActor = VerifyActor (Mailbox VerifyMessage)

-- | Start the actor; it lives as long as the continuation. A failed GPU
-- call never reaches 'link': 'verifyWithPolicy' catches 'VerifierException'.
withVerifyActor :: (MonadUnliftIO m, MonadLoggerIO m) => VerifyConfig -> (VerifyActor -> m a) -> m a
withVerifyActor cfg action = do
  (inbox, mailbox) <- newMailbox
  $(logDebugS) "Verify" "Starting verify actor"
  withAsync (run inbox Nothing) $ \a -> link a >> action (VerifyActor mailbox)
  where
    -- held: what was taken from the mailbox while a tx batch was formed and
    -- did not fit it (a block, or a tx past maxInputs); it is handled next
    run inbox held = do
      p <- maybe (PendingMsg <$> receive inbox) return held
      case p of
        PendingMsg (VerifyBlock b) -> handleBlock b >> run inbox Nothing
        PendingMsg (VerifyTx t) -> liftIO (cfg.txPrevouts t) >>= batchFrom inbox t
        PendingTx t ins -> batchFrom inbox t ins
    batchFrom inbox t ins = do
      t0 <- liftIO getMonotonicTimeNSec
      (batch, held') <- collect inbox t0 [(t, ins)] (length ins)
      handleTxs batch
      run inbox held'
    -- coalesce VerifyTx messages: drain the mailbox until the batch holds
    -- maxInputs inputs or maxWaitMicros have passed since its first tx
    collect inbox t0 acc n
      | n >= cfg.maxInputs = return (reverse acc, Nothing)
      | otherwise = do
          now <- liftIO getMonotonicTimeNSec
          let left = cfg.maxWaitMicros - fromIntegral ((now - t0) `div` 1000)
          mm <- if left <= 0 then return Nothing else timeout left (receive inbox)
          case mm of
            Nothing -> return (reverse acc, Nothing)
            Just (VerifyTx t) -> do
              ins <- liftIO (cfg.txPrevouts t)
              if n + length ins > cfg.maxInputs
                then return (reverse acc, Just (PendingTx t ins))
                else collect inbox t0 ((t, ins) : acc) (n + length ins)
            Just other -> return (reverse acc, Just (PendingMsg other))
    handleBlock b = do
      ins <- liftIO (cfg.prevouts b)
      let h = headerHash b.header
      ok <- verifyWithPolicy cfg b.txs ins
      let bad = [(t, i) | ((t, i, _, _), False) <- zip ins ok]
      if null bad
        then publish (BlockVerified h) cfg.pub
        else do
          $(logWarnS) "Verify" "Block has inputs that fail verifyStdInput"
          publish (BlockRejected h bad) cfg.pub
    -- one GPU call for the whole coalesced batch: tx k of the batch is tx
    -- index k of the call
    handleTxs batch = do
      let txs = map fst batch
          ins = [(k, i, so, val) | (k, (_, xs)) <- zip [0 ..] batch, (i, so, val) <- xs]
      ok <- if null ins then return [] else verifyWithPolicy cfg txs ins
      -- the verdicts in batch order, cut per tx (one pass)
      forM_ (zip batch (splitPlaces (map (length . snd) batch) ok)) $ \((t, xs), vs) -> do
        let bad = [i | ((i, _, _), False) <- zip xs vs]
        publish (if null bad then TxVerified (txHash t) else TxRejected (txHash t) bad) cfg.pub
    splitPlaces [] _ = []
    splitPlaces (c : cs) xs = let (a, b) = splitAt c xs in a : splitPlaces cs b

-- | What the actor handles next: a message from the mailbox, or a tx whose
-- prevouts were looked up while a batch was formed that it did not fit.
data Pending
  = PendingMsg !VerifyMessage
  | PendingTx !Tx ![(Int, ScriptOutput, Word64)]

-- | The error policy (SURVEY.md §5 failure detection): a failed GPU call
-- (any 'VerifierException': HKV_E_INTERNAL when the call's multisig tail
-- gave up, a device error) is re-submitted up to 'retries' times; then the
-- batch is re-verified on the CPU with haskoin-core's own per-input
-- 'verifyStdInput' (the path the drop-in replaces). Nothing is thrown, so
-- 'link' never takes the node down for a verify failure.
verifyWithPolicy ::
  (MonadUnliftIO m, MonadLoggerIO m) => VerifyConfig -> [Tx] -> [(Int, Int, ScriptOutput, Word64)] -> m [Bool]
verifyWithPolicy cfg txs ins = attempt (cfg.retries + 1)
  where
    attempt k = do
      r <- liftIO (try (verifyStdInputBatch cfg.verifier cfg.net txs ins))
      case r of
        Right ok -> return ok
        Left (VerifierException msg rc) -> do
          $(logWarnS) "Verify" ("GPU batch failed (" <> T.pack msg <> ", rc " <> T.pack (show rc) <> ")")
          if k > 1 then attempt (k - 1) else cpu
    arr = listArray (0, length txs - 1) txs
    cpu = do
      $(logWarnS) "Verify" "Re-verifying the batch on the CPU (verifyStdInput)"
      return [verifyStdInput cfg.net cfg.secp (arr ! t) i so val | (t, i, so, val) <- ins]

-- | Forward a block from PeerEvent (PeerMessage _ (MBlock b)) (Node.hs:172).
verifyBlock :: (MonadIO m) => Block -> VerifyActor -> m ()
verifyBlock b (VerifyActor mb) = VerifyBlock b `send` mb

-- | Forward a transaction from PeerEvent (PeerMessage _ (MTx t)).
verifyTx :: (MonadIO m) => Tx -> VerifyActor -> m ()
verifyTx t (VerifyActor mb) = VerifyTx t `send` mb

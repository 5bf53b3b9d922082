{-# LANGUAGE ForeignFunctionInterface #-}

-- | Raw bindings to libhkv's C ABI (include/hkv.h), the MI355X batch
-- verifier. UNCOMPILED in this repository's image (no GHC): written against
-- include/hkv.h and checked only by reading; the same ABI is exercised from
-- Python (haskoin-node_amd/hkv/lib.py mirrors these signatures one for one,
-- tests/test_abi.py checks every exported symbol).
--
-- Replaces, one batch at a time, the per-signature FFI of
-- secp256k1-haskell-1.2.0 (pinned /root/reference/stack.yaml:9):
-- @secp256k1_ecdsa_verify@ behind @verifySig@, and haskoin-core-1.1.0's
-- @verifyHashSig@ (stack.yaml:10) through mode 'hkvHaskoin'.
module Haskoin.Node.Verify.FFI
  ( HkvCtx,
    HkvBatch,
    HkvTxs (..),
    InputJob (..),
    c_hkv_open,
    c_hkv_close,
    c_hkv_batch_alloc,
    c_hkv_batch_free,
    c_hkv_batch_records,
    c_hkv_batch_capacity,
    c_hkv_verify,
    c_hkv_verify_std_inputs,
    c_hkv_verify_std_inputs_device_status,
    c_hkv_device_fault,
    c_hkv_device_healthy,
    c_hkv_check_headers,
    c_hkv_merkle_roots,
    c_hkv_strerror,
    hkvLibsecp,
    hkvHaskoin,
    hkvRecordSize,
    hkvNoForkId,
    hkvEInternal,
    hkvStatusTailFault,
  )
where

import Data.Int (Int32)
import Data.Word (Word32, Word64, Word8)
import Foreign.C.String (CString)
import Foreign.C.Types (CInt (..), CSize (..))
import Foreign.Ptr (Ptr)
import Foreign.Storable (Storable (..))

-- | Opaque handles (struct hkv_ctx, struct hkv_batch).
data HkvCtx

data HkvBatch

-- | struct hkv_txs: serialised txs back to back, n_tx + 1 byte offsets and a
-- pool of prevout scripts (include/hkv.h). 40 bytes on x86-64.
data HkvTxs = HkvTxs
  { txsBytes :: !(Ptr Word8),
    txsOffsets :: !(Ptr Word32),
    txsCount :: !Word32,
    txsScripts :: !(Ptr Word8),
    txsScriptsLen :: !Word32
  }

instance Storable HkvTxs where
  sizeOf _ = 40
  alignment _ = 8
  peek p =
    HkvTxs
      <$> peekByteOff p 0
      <*> peekByteOff p 8
      <*> peekByteOff p 16
      <*> peekByteOff p 24
      <*> peekByteOff p 32
  poke p t = do
    pokeByteOff p 0 (txsBytes t)
    pokeByteOff p 8 (txsOffsets t)
    pokeByteOff p 16 (txsCount t)
    pokeByteOff p 24 (txsScripts t)
    pokeByteOff p 32 (txsScriptsLen t)

-- | struct hkv_input_job (24 bytes): input @input@ of tx @tx@ spends a prevout
-- whose scriptPubKey is scripts[script_off, +script_len) and amount @value@.
data InputJob = InputJob
  { jobTx :: !Word32,
    jobInput :: !Word32,
    jobScriptOff :: !Word32,
    jobScriptLen :: !Word32,
    jobValue :: !Word64
  }

instance Storable InputJob where
  sizeOf _ = 24
  alignment _ = 8
  peek p =
    InputJob
      <$> peekByteOff p 0
      <*> peekByteOff p 4
      <*> peekByteOff p 8
      <*> peekByteOff p 12
      <*> peekByteOff p 16
  poke p j = do
    pokeByteOff p 0 (jobTx j)
    pokeByteOff p 4 (jobInput j)
    pokeByteOff p 8 (jobScriptOff j)
    pokeByteOff p 12 (jobScriptLen j)
    pokeByteOff p 16 (jobValue j)

hkvLibsecp, hkvHaskoin :: Word32
hkvLibsecp = 0 -- secp256k1_ecdsa_verify: high-S rejected

hkvHaskoin = 1 -- verifyHashSig: normalizeSig, then verify

hkvRecordSize :: Int
hkvRecordSize = 168 -- msg32 | r | s | pklen | pubkey[65] | pad[6]

hkvNoForkId :: Int32
hkvNoForkId = -1

-- | HKV_E_INTERNAL: what hkv_verify_std_inputs returns when its own call's
-- multisig tail reported HKV_STATUS_TAIL_FAULT (some multisig verdicts were
-- left at 0); the actor re-submits the batch (Verify.hs verifyWithPolicy).
hkvEInternal :: CInt
hkvEInternal = -5

-- | HKV_STATUS_TAIL_FAULT, the bit the _status form and hkv_device_fault report.
hkvStatusTailFault :: Word32
hkvStatusTailFault = 1

-- Context / batch lifetime: cheap, may use `unsafe`.
foreign import ccall safe "hkv_open"
  c_hkv_open :: CInt -> Word32 -> Ptr (Ptr HkvCtx) -> IO CInt

foreign import ccall safe "hkv_close"
  c_hkv_close :: Ptr HkvCtx -> IO ()

foreign import ccall unsafe "hkv_batch_alloc"
  c_hkv_batch_alloc :: Ptr HkvCtx -> CSize -> Ptr (Ptr HkvBatch) -> IO CInt

foreign import ccall unsafe "hkv_batch_free"
  c_hkv_batch_free :: Ptr HkvBatch -> IO ()

foreign import ccall unsafe "hkv_batch_records"
  c_hkv_batch_records :: Ptr HkvBatch -> IO (Ptr Word8)

foreign import ccall unsafe "hkv_batch_capacity"
  c_hkv_batch_capacity :: Ptr HkvBatch -> IO CSize

-- The GPU calls block for milliseconds: `safe` releases the capability so
-- other Haskell threads run meanwhile (needs the -threaded RTS).
foreign import ccall safe "hkv_verify"
  c_hkv_verify :: Ptr HkvCtx -> Ptr HkvBatch -> CSize -> Word32 -> Ptr Word32 -> IO CInt

foreign import ccall safe "hkv_verify_std_inputs"
  c_hkv_verify_std_inputs :: Ptr HkvCtx -> Ptr HkvTxs -> Ptr InputJob -> CSize -> Int32 -> Ptr Word32 -> IO CInt

-- The asynchronous block path: everything is enqueued on the caller's HIP
-- stream (the last argument); d_status gets HKV_STATUS_* bits ORed in on it.
foreign import ccall safe "hkv_verify_std_inputs_device_status"
  c_hkv_verify_std_inputs_device_status ::
    Ptr HkvCtx -> CInt -> Ptr HkvTxs -> Ptr InputJob -> CSize -> Int32 -> Ptr () -> Ptr Word32 -> Ptr Word32 ->
    Ptr () -> IO CInt

-- Read and clear device dev's sticky fault latch (waits for its enqueued calls).
foreign import ccall safe "hkv_device_fault"
  c_hkv_device_fault :: Ptr HkvCtx -> CInt -> Ptr Word32 -> IO CInt

foreign import ccall unsafe "hkv_device_healthy"
  c_hkv_device_healthy :: Ptr HkvCtx -> CInt -> IO CInt

foreign import ccall safe "hkv_check_headers"
  c_hkv_check_headers ::
    Ptr HkvCtx -> Ptr Word8 -> CSize -> Ptr Word8 -> Ptr Word8 -> Ptr Word8 -> Ptr Word8 -> IO CInt

foreign import ccall safe "hkv_merkle_roots"
  c_hkv_merkle_roots :: Ptr HkvCtx -> Ptr Word8 -> Ptr Word32 -> CSize -> Ptr Word8 -> Ptr Word8 -> IO CInt

foreign import ccall unsafe "hkv_strerror"
  c_hkv_strerror :: CInt -> IO CString

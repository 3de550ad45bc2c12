//! The drop-in test, following zarrs/tests/codec_runtime_registration.rs:92-183: an array written by
//! zarrs' own (CPU) sharding encoder is reopened with the GPU `sharding_indexed` plugin registered,
//! and every read (whole array, partial shards, one element, the batched array extension) must equal
//! what zarrs reads without the plugin. Needs a GPU (HIP device ZARRS_GPU_DEVICE, default 0).

use std::sync::Arc;

use zarrs::array::{Array, ArrayBuilder, ArraySubset, codec, data_type};
use zarrs::storage::store::MemoryStore;
use zarrs_gpu::ArrayGpuExt;

fn write_array(store: Arc<MemoryStore>) -> Vec<u16> {
    let array = ArrayBuilder::new(vec![64, 96], vec![32, 48], data_type::uint16(), 7u16)
        .subchunk_shape(vec![8, 16])
        .bytes_to_bytes_codecs(vec![
            Arc::new(codec::GzipCodec::new(1).unwrap()),
            Arc::new(codec::Crc32cCodec::new()),
        ])
        .build(store, "/array")
        .unwrap();
    array.store_metadata().unwrap();
    let data: Vec<u16> = (0..64 * 96).map(|i| ((i * 37) % 4001) as u16).collect();
    array.store_array_subset(&array.subset_all(), &data).unwrap();
    data
}

#[test]
fn gpu_sharding_plugin_matches_zarrs() {
    let store = Arc::new(MemoryStore::default());
    let data = write_array(store.clone());
    let subsets = [
        ArraySubset::new_with_ranges(&[0..64, 0..96]),  // whole shards: decode_into, crc32c verified
        ArraySubset::new_with_ranges(&[5..40, 17..90]), // partial shards: the partial decoder
        ArraySubset::new_with_ranges(&[33..34, 50..51]), // one element
    ];
    let cpu: Array<MemoryStore> = Array::open(store.clone(), "/array").unwrap();
    let expected: Vec<Vec<u16>> = subsets.iter().map(|s| cpu.retrieve_array_subset(s).unwrap()).collect();
    assert_eq!(expected[0], data);

    let handle = zarrs_gpu::register();
    let gpu: Array<MemoryStore> = Array::open(store.clone(), "/array").unwrap();
    for (s, e) in subsets.iter().zip(&expected) {
        let got: Vec<u16> = gpu.retrieve_array_subset(s).unwrap();
        assert_eq!(&got, e);
        // the batched extension (all shards of the subset in one call)
        let raw = gpu.retrieve_array_subset_gpu(s).unwrap();
        let got2: Vec<u16> = raw.chunks_exact(2).map(|b| u16::from_ne_bytes([b[0], b[1]])).collect();
        assert_eq!(&got2, e);
    }
    assert!(zarrs_gpu::unregister(&handle));
    assert!(!zarrs_gpu::unregister(&handle));
}

#[test]
fn gpu_multi_device_read_matches_zarrs() {
    // devices [0, 0] on a one-GPU machine: two contexts of one device still exercise the split
    let store = Arc::new(MemoryStore::default());
    let _ = write_array(store.clone());
    let cpu: Array<MemoryStore> = Array::open(store.clone(), "/array").unwrap();
    let subset = ArraySubset::new_with_ranges(&[3..61, 7..95]);
    let expected: Vec<u16> = cpu.retrieve_array_subset(&subset).unwrap();
    let raw = cpu.retrieve_array_subset_gpu_multi(&subset, &[0, 0]).unwrap();
    let got: Vec<u16> = raw.chunks_exact(2).map(|b| u16::from_ne_bytes([b[0], b[1]])).collect();
    assert_eq!(got, expected);
}

/// Unsharded arrays through zarrs' unchanged per-chunk read path with the per-codec GPU plugins
/// registered (transpose + big-endian bytes: config C2's chain; bytes + shuffle + zstd: C5's;
/// bytes + gzip + crc32c), against the same reads without them.
#[test]
fn gpu_per_codec_plugins_match_zarrs() {
    let store = Arc::new(MemoryStore::default());
    let chains = ["/c2", "/c5", "/gz"];
    for path in &chains {
        let mut b = ArrayBuilder::new(vec![40, 70, 33], vec![16, 32, 16], data_type::uint16(), 3u16);
        match *path {
            "/c2" => {
                b.array_to_array_codecs(vec![Arc::new(codec::TransposeCodec::new(
                    codec::TransposeOrder::new(&[2, 1, 0]).unwrap(),
                ))])
                .array_to_bytes_codec(Arc::new(codec::BytesCodec::big()));
            }
            "/c5" => {
                b.bytes_to_bytes_codecs(vec![
                    Arc::new(codec::ShuffleCodec::new(2)),
                    Arc::new(codec::ZstdCodec::new(3, false)),
                ]);
            }
            _ => {
                b.bytes_to_bytes_codecs(vec![
                    Arc::new(codec::GzipCodec::new(1).unwrap()),
                    Arc::new(codec::Crc32cCodec::new()),
                ]);
            }
        }
        let array = b.build(store.clone(), path).unwrap();
        array.store_metadata().unwrap();
        let data: Vec<u16> = (0..40 * 70 * 33).map(|i| ((i * 7919) % 5003) as u16).collect();
        array.store_array_subset(&array.subset_all(), &data).unwrap();
    }
    let subsets = [
        ArraySubset::new_with_ranges(&[0..40, 0..70, 0..33]),
        ArraySubset::new_with_ranges(&[3..37, 10..65, 5..30]),
    ];
    let expected: Vec<Vec<Vec<u16>>> = chains
        .iter()
        .map(|p| {
            let a: Array<MemoryStore> = Array::open(store.clone(), p).unwrap();
            subsets.iter().map(|s| a.retrieve_array_subset(s).unwrap()).collect()
        })
        .collect();
    // the entropy stages on the GPU (the default), then every stage
    for register in [zarrs_gpu::register_codecs, zarrs_gpu::register_codecs_all] {
        let handle = register();
        for (p, exp) in chains.iter().zip(&expected) {
            let a: Array<MemoryStore> = Array::open(store.clone(), p).unwrap();
            for (s, e) in subsets.iter().zip(exp) {
                let got: Vec<u16> = a.retrieve_array_subset(s).unwrap();
                assert_eq!(&got, e, "{p}");
            }
        }
        assert!(zarrs_gpu::unregister(&handle));
    }
}

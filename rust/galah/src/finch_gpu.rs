//! finch::distances (src/finch.rs:26-75) on MI355X GPUs through
//! libgalahgpu.so (galah-gpu-sys).  Built with `--features gpu`; the
//! signature, the FinchPreclusterer struct and trait impl (src/finch.rs:4-24)
//! and the Preclusterer::Finch construction (CAP:959-982) are unchanged, and
//! finch::distances calls this body when the feature is on.
//!
//! Output: the same SortedPairGenomeDistanceCache -- (i, j) with i < j for
//! every pair with 1 - mash_distance >= min_ani as f64, stored as
//! Some(ani as f32) (src/finch.rs:56-71).  At debug level every compared pair
//! is logged with src/finch.rs:65-68's line, in the reference's loop order,
//! streamed from the library in row blocks (gg_precluster_files_each) so the
//! N(N-1)/2 pairs are never held at once.
use crate::sorted_pair_genome_distance_cache::SortedPairGenomeDistanceCache;
use galah_gpu_sys::*;
use std::ffi::{CStr, CString};
use std::os::raw::{c_char, c_int, c_void};

/// What the debug line of a compared pair needs (the sink's `user`).
struct ComparedPairs<'a> {
    paths: &'a [&'a str],
    kmer_length: c_int,
}

/// gg_pair_sink: src/finch.rs:65-68 for each pair of a block.
unsafe extern "C" fn log_compared(user: *mut c_void, pairs: *const gg_pair, n: u64) -> c_int {
    let c = &*(user as *const ComparedPairs);
    if n == 0 {
        return 0;
    }
    for p in std::slice::from_raw_parts(pairs, n as usize) {
        // 1 - finch mash_distance(common, total) in f64, the value the
        // reference prints
        let distance = gg_ani_f64(p.common, p.total, c.kmer_length);
        debug!(
            "Comparing {} and {}, distance {}",
            c.paths[p.i as usize], c.paths[p.j as usize], distance
        );
    }
    0
}

unsafe fn failure(ctx: *mut gg_ctx) -> String {
    let msg = CStr::from_ptr(gg_last_error(ctx)).to_string_lossy().into_owned();
    gg_destroy(ctx);
    msg
}

pub fn distances(
    genome_fasta_paths: &[&str],
    min_ani: f32,
    num_kmers: usize,
    kmer_length: u8,
) -> SortedPairGenomeDistanceCache {
    info!("Sketching MinHash representations of each genome with finch ..");
    let c_paths: Vec<CString> = genome_fasta_paths
        .iter()
        .map(|p| CString::new(*p).expect("Failed to sketch genomes with finch"))
        .collect();
    let ptrs: Vec<*const c_char> = c_paths.iter().map(|c| c.as_ptr()).collect();
    let mut to_return = SortedPairGenomeDistanceCache::new();
    unsafe {
        let mut st: GgStatus = GG_OK;
        // every visible GPU (or GALAHGPU_DEVICES); one host thread per GPU
        // inside the library
        let ctx = gg_create_multi(kmer_length as c_int, num_kmers as u32, 0, std::ptr::null(), 0, &mut st);
        if ctx.is_null() {
            panic!(
                "Failed to sketch genomes with finch: {}",
                CStr::from_ptr(gg_thread_last_error()).to_string_lossy()
            );
        }
        // file ingest on galah's --threads: the global rayon pool (CAP:408-412)
        gg_set_host_threads(ctx, rayon::current_num_threads() as c_int);
        let (mut pairs, mut ani, mut n) = (std::ptr::null_mut(), std::ptr::null_mut(), 0u64);
        let status = if log_enabled!(log::Level::Debug) {
            let compared = ComparedPairs {
                paths: genome_fasta_paths,
                kmer_length: kmer_length as c_int,
            };
            gg_precluster_files_each(
                ctx,
                ptrs.as_ptr(),
                ptrs.len() as u32,
                min_ani,
                std::ptr::null(),
                Some(log_compared),
                &compared as *const ComparedPairs as *mut c_void,
                &mut pairs,
                &mut ani,
                &mut n,
                std::ptr::null_mut(),
            )
        } else {
            gg_precluster_files(ctx, ptrs.as_ptr(), ptrs.len() as u32, min_ani, &mut pairs, &mut ani, &mut n)
        };
        if status != GG_OK {
            panic!("Failed to sketch genomes with finch: {}", failure(ctx)); // src/finch.rs:50
        }
        info!("Finished sketching genomes");
        // device count, phase times and any slow path taken (gg_info_line)
        let mut line = [0 as c_char; 1024];
        if gg_info_line(ctx, line.as_mut_ptr(), line.len()) == GG_OK {
            info!("{}", CStr::from_ptr(line.as_ptr()).to_string_lossy());
        }
        if n > 0 {
            let p = std::slice::from_raw_parts(pairs, n as usize);
            let a = std::slice::from_raw_parts(ani, n as usize);
            for (x, v) in p.iter().zip(a) {
                // Some(ani as f32) of 1 - mash_distance in f64 (src/finch.rs:56-70)
                to_return.insert((x.i as usize, x.j as usize), Some(*v));
            }
        }
        gg_free(pairs as *mut c_void);
        gg_free(ani as *mut c_void);
        gg_destroy(ctx);
    }
    to_return
}

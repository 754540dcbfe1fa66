# PamgHIPPartitionedArraysExt — PartitionedArrays.jl (v0.5 API) adapter of PamgHIP.
#
# NOT EXECUTED: Julia and PartitionedArrays.jl are absent from this image and from the GPU
# boxes (no network). tests/test_julia_binding.py checks statically that every ccall matches
# include/pamg.h and that every method below extends PartitionedArrays' / LinearAlgebra's /
# Base's own generic function (no PamgHIP generic of the same name exists). The PartitionedArrays
# calls used (partition, own_to_local, ghost_to_local, ghost_to_owner, local_to_global,
# global_to_local, own_own_values, own_ghost_values, ExchangeGraph, exchange, JaggedArray,
# gather, reduction, linear_indices) are written against the v0.5 documentation and are
# unverified here.
#
# An AMG solver written against PartitionedArrays keeps calling mul!, consistent!, dot, norm,
# axpy!, ldiv!, own_values on PSparseMatrix / PVector; this extension moves the parts onto the
# GPU(s) once and gives those generic functions device methods that run libpamg's kernels:
#
#   A_d = hip(ctxs, A)            # PSparseMatrix -> HIPPSparseMatrix (one DeviceMatrix per part)
#   x_d = hip(ctxs, x)            # PVector       -> HIPPVector       (own + ghost slots per part)
#   M   = HIPPVCycle(ctxs, A)     # distributed SA setup (SPEC §S4/§S7) + device V-cycle per part
#   mul!(y_d, A_d, x_d)           # ghost exchange (RCCL / debug transport) + SpMV per part
#   t = consistent!(x_d); wait(t) # split exchange (pamg_exchange_begin / _end); t is a Task
#   ldiv!(z_d, M, r_d)            # one V-cycle from zero (the Pl = M preconditioner)
#   copyto!(x, x_d)               # own values back into the PartitionedArrays vector
#
# `ctxs` is a PartitionedArrays array of PamgHIP.Context, one per part, made with `map` over
# the parts:
#   with_mpi:   one rank = one part = one GPU, each context comm_init!'ed (RCCL);
#   with_debug: all parts in one process — the contexts of one PamgHIP.World,
#               `w = World(nparts); ctxs = map(p -> w.ctxs[p], LinearIndices((nparts,)))`
#               (libpamg's in-process transport: ghosts copied device to device from the
#               sibling parts' vectors; parts may share one GPU). A part's exchange waits for its
#               neighbours' inside the library, so the methods below run every exchanging
#               operation (mul!, consistent!, dot, ldiv!) for all parts in ONE call
#               (world_spmv!, world_exchange!, world_dot, world_vcycle!: a thread per part
#               inside libpamg) instead of a sequential map; local operations stay a map.
#
# Layout mapping. PartitionedArrays numbers a part's local indices own-first for the
# OwnAndGhostIndices it builds (uniform_partition + ghosts), with ghosts in the order of
# ghost_to_global. libpamg wants the ghosts grouped by owner, in neighbour order (SPEC §S7,
# include/pamg.h pamg_plan_create). `DeviceLayout` records the permutation: device ghost slot
# j holds PartitionedArrays local index `ghost_lids[j]`; matrix columns are renumbered with it
# at upload and vectors are permuted on the way in and out. Send lists are the owners' local
# indices of the ghosts each neighbour holds, obtained with PartitionedArrays' own `exchange`.
module PamgHIPPartitionedArraysExt

using LinearAlgebra
using SparseArrays
using PartitionedArrays
using PamgHIP
import PamgHIP: DeviceVector, DeviceMatrix, ExchangePlan, Context, HostCSR

# ------------------------------------------------------------------ messages between parts
# The backend.exchange / allgather / allreduce_max of parallel_amg_amd/backend.py, on
# PartitionedArrays' own collectives, so the setup driver below reads like hierarchy.py.

"Per part a Dict(dest part => payload vector); returns per part a Dict(src part => payload)."
function _exchange(msgs, ::Type{T}) where {T}
    snd = map(d -> sort!(collect(keys(d))), msgs)
    graph = ExchangeGraph(snd)                       # discovers the receivers
    data = map((d, s) -> JaggedArray([Vector{T}(d[k]) for k in s]), msgs, snd)
    rcv = fetch(exchange(data, graph))
    map((r, srcs) -> Dict(zip(srcs, [collect(r[i]) for i in 1:length(srcs)])), rcv, graph.rcv)
end
_allgather(vals) = gather(vals; destination = :all)
_allreduce_max(vals) = reduction(max, vals; destination = :all, init = -Inf)

# ------------------------------------------------------------------ layout of one part
struct DeviceLayout
    n_own::Int
    own_lids::Vector{Int32}       # PartitionedArrays local ids of the own entries, device order
    ghost_lids::Vector{Int32}     # ... of the ghost entries, device slot order
    lid_to_device::Vector{Int32}  # PartitionedArrays local id -> device local id (1-based)
    nbr_ranks::Vector{Int32}      # 0-based ranks, device neighbour order
    recv_counts::Vector{Int64}
end

function device_layout(ids)
    own = Int32.(collect(own_to_local(ids)))
    gl = collect(ghost_to_local(ids))
    owner = collect(ghost_to_owner(ids))
    # ghosts grouped by owner (ascending part id), original order within a group (stable)
    perm = sortperm(owner; alg = Base.Sort.DEFAULT_STABLE)
    ghost_lids = Int32.(gl[perm])
    nbrs = unique(owner[perm])
    counts = Int64[count(==(q), owner) for q in nbrs]
    l2d = zeros(Int32, local_length(ids))
    for (k, l) in enumerate(own)
        l2d[l] = k
    end
    for (k, l) in enumerate(ghost_lids)
        l2d[l] = length(own) + k
    end
    DeviceLayout(length(own), own, ghost_lids, l2d, Int32.(nbrs .- 1), counts)
end

"""
Per-part exchange plans for the index partition `rows` (a PRange's `partition`): each part
asks the owners of its ghosts (in device order) for them, and the requests an owner receives
are its send lists. Neighbour lists are the union of both directions (a part may only send to,
or only receive from, another), as pamg_plan_create allows.
"""
function exchange_plans(ctxs, rows, layouts)
    reqs = map(rows, layouts) do ids, lay
        g = local_to_global(ids)
        d = Dict{Int,Vector{Int64}}()
        off = 0
        for (q, c) in zip(lay.nbr_ranks, lay.recv_counts)
            d[Int(q) + 1] = Int64[g[lay.ghost_lids[off + i]] for i in 1:c]
            off += c
        end
        d
    end
    got = _exchange(reqs, Int64)
    map(ctxs, rows, layouts, got) do ctx, ids, lay, req
        g2l = global_to_local(ids)
        nbrs = sort!(union(Int.(lay.nbr_ranks) .+ 1, collect(keys(req))))
        rc = Dict(zip(Int.(lay.nbr_ranks) .+ 1, lay.recv_counts))
        send_idx = Int64[]
        send_counts = Int64[]
        for q in nbrs
            lst = get(req, q, Int64[])
            push!(send_counts, length(lst))
            append!(send_idx, (lay.lid_to_device[g2l[gid]] for gid in lst))  # device own index (1-based)
        end
        ExchangePlan(ctx, lay.n_own, sum(lay.recv_counts; init = 0), Int32.(nbrs .- 1),
                     Int64[get(rc, q, 0) for q in nbrs], send_counts, send_idx)
    end
end

# ------------------------------------------------------------------ distributed wrappers
struct HIPPVector{A,B,C}
    parts::A     # DeviceVector per part
    layouts::B   # DeviceLayout per part
    plans::C     # ExchangePlan per part
end
struct HIPPSparseMatrix{A,B,C}
    parts::A     # DeviceMatrix per part
    col_layouts::B
    plans::C
end

PartitionedArrays.partition(x::HIPPVector) = x.parts
PartitionedArrays.partition(A::HIPPSparseMatrix) = A.parts
"own_values(x): per part, the own values (host copies, PartitionedArrays' own order)."
PartitionedArrays.own_values(x::HIPPVector) =
    map(PamgHIP.download_own, x.parts)   # device own order = own_to_local order
"ghost_values(x): per part, the ghost slots as last exchanged, in PartitionedArrays' ghost order."
PartitionedArrays.ghost_values(x::HIPPVector) =
    map(x.parts, x.layouts) do dv, lay
        gd = PamgHIP.download_ghosts(dv)                     # device slot order (grouped by owner)
        gl = lay.ghost_lids .- lay.n_own                      # PartitionedArrays ghost position
        out = similar(gd)
        out[gl] .= gd
        out
    end

"Upload a PVector (own values; ghosts come with the next consistent!)."
function PamgHIP.hip(ctxs, x::PVector; plans = nothing)
    rows = partition(axes(x, 1))
    layouts = map(device_layout, rows)
    plans = plans === nothing ? exchange_plans(ctxs, rows, layouts) : plans
    dv = map(ctxs, partition(x), layouts) do ctx, vals, lay
        PamgHIP.DeviceVector(ctx, vals[lay.own_lids], sum(lay.recv_counts; init = 0))
    end
    HIPPVector(dv, layouts, plans)
end

"""
One part's own rows as 0-based-free CSR arrays in the device column layout: PartitionedArrays
v0.5 stores a part's local matrix in split format, so the own rows are the own-own block
(columns = own positions) beside the own-ghost block (columns = ghost positions); each row is
merged in ascending GLOBAL column order (SPEC §S1).
"""
function _own_rows_csr(Aoo::SparseMatrixCSC, Aog::SparseMatrixCSC, cids, lay::DeviceLayout)
    cg = local_to_global(cids)
    own_l = collect(own_to_local(cids))                 # own position k -> local id
    gh_l = collect(ghost_to_local(cids))                # ghost position k -> local id
    To, Tg = sparse(transpose(Aoo)), sparse(transpose(Aog))   # column j = own row j
    n = size(To, 2)
    rowptr = ones(Int64, n + 1)
    colv, valv = Int64[], Float64[]
    for j in 1:n
        ro = To.colptr[j]:(To.colptr[j+1]-1)
        rg = Tg.colptr[j]:(Tg.colptr[j+1]-1)
        lids = vcat(own_l[To.rowval[ro]], gh_l[Tg.rowval[rg]])
        vals = vcat(To.nzval[ro], Tg.nzval[rg])
        o = sortperm(cg[lids])
        append!(colv, lay.lid_to_device[lids[o]])
        append!(valv, vals[o])
        rowptr[j+1] = length(colv) + 1
    end
    rowptr, colv, valv
end

"Upload a PSparseMatrix: own rows, columns renumbered into the device column layout."
function PamgHIP.hip(ctxs, A::PSparseMatrix)
    rows = partition(axes(A, 1))
    cols = partition(axes(A, 2))
    clay = map(device_layout, cols)
    plans = exchange_plans(ctxs, cols, clay)
    dm = map(ctxs, own_own_values(A), own_ghost_values(A), cols, clay, plans) do ctx, Aoo, Aog, cids, lay, plan
        rowptr, colv, valv = _own_rows_csr(Aoo, Aog, cids, lay)
        PamgHIP.DeviceMatrix(ctx, rowptr, colv, valv, lay.n_own + sum(lay.recv_counts; init = 0);
                             plan = isempty(lay.nbr_ranks) ? nothing : plan, index_base = 1)
    end
    HIPPSparseMatrix(dm, clay, plans)
end

"Own values back into the PartitionedArrays vector."
function Base.copyto!(x::PVector, xd::HIPPVector)
    map(partition(x), xd.parts, xd.layouts) do vals, dv, lay
        vals[lay.own_lids] .= PamgHIP.download_own(dv)
    end
    x
end

Base.similar(x::HIPPVector) = HIPPVector(map(similar, x.parts), x.layouts, x.plans)

# the World of a debug-backend distribution (every part's context in one), or nothing
function _world(parts)
    ps = collect(parts)
    w = first(ps).ctx.world
    (w === nothing || length(ps) < 2) && return nothing
    w
end

function LinearAlgebra.mul!(y::HIPPVector, A::HIPPSparseMatrix, x::HIPPVector)
    w = _world(x.parts)
    w === nothing ? foreach(mul!, y.parts, A.parts, x.parts) :
        PamgHIP.world_spmv!(w, collect(y.parts), collect(A.parts), collect(x.parts))
    y
end

"""
consistent!(x): PartitionedArrays' contract — start the ghost exchange and return a task;
`wait(t)` (or `fetch`) completes it and yields x. Every part's exchange is enqueued here, on the
part's comm stream (pamg_exchange_begin); the Task joins them (pamg_exchange_end).
"""
function PartitionedArrays.consistent!(x::HIPPVector)
    w = _world(x.parts)
    if w !== nothing  # in-process transport: synchronous, all parts in one call
        PamgHIP.world_exchange!(w, collect(x.parts), collect(x.plans))
        return @async x
    end
    tasks = map(PamgHIP.exchange_begin, x.parts, x.plans)
    @async begin
        foreach(wait, tasks)
        x
    end
end

# Reductions: every part's pamg_vec_dot returns the global sum (the all-reduce inside libpamg:
# RCCL, or the in-process world's rank-order sum, which is collective — all parts in one call).
function LinearAlgebra.dot(x::HIPPVector, y::HIPPVector)
    w = _world(x.parts)
    w === nothing || return PamgHIP.world_dot(w, collect(x.parts), collect(y.parts))
    getany(map(dot, x.parts, y.parts))
end
LinearAlgebra.norm(x::HIPPVector) = sqrt(dot(x, x))
LinearAlgebra.axpy!(a::Real, x::HIPPVector, y::HIPPVector) = (foreach((xp, yp) -> axpy!(a, xp, yp), x.parts, y.parts); y)
LinearAlgebra.axpby!(a::Real, x::HIPPVector, b::Real, y::HIPPVector) =
    (foreach((xp, yp) -> axpby!(a, xp, b, yp), x.parts, y.parts); y)
Base.fill!(x::HIPPVector, v::Real) = (foreach(p -> fill!(p, v), x.parts); x)
Base.copy!(d::HIPPVector, s::HIPPVector) = (foreach(copy!, d.parts, s.parts); d)

# ------------------------------------------------------------------ distributed setup driver
# parallel_amg_amd/hierarchy.py's build_hierarchy in PartitionedArrays terms: per-part C-ABI
# setup kernels (PamgHIP.gershgorin / aggregate / tentative / spgemm / smooth / transpose_piece)
# separated by exchanges of ghost rows, so every part ends with the rows the global-view oracle
# gives it (SPEC §S4.5, §S7). Row ids are global and 0-based, as in the C-ABI.

"A part's ghost plan of a column space: ghost global ids (ascending) and the exchange lists."
struct HostPlan
    n_own::Int
    col0::Int
    ghost_ids::Vector{Int64}
    nbrs::Vector{Int}             # 1-based parts, ascending
    recv_counts::Vector{Int64}
    send_counts::Vector{Int64}
    send_idx::Vector{Int64}       # 0-based own indices, concatenated per neighbour
    sends::Dict{Int,Vector{Int64}}
end

_owner(ids, offs) = searchsortedlast.(Ref(offs), ids)       # 1-based part of 0-based global ids

function _ghost_ids(M::HostCSR, lo::Integer, hi::Integer)
    _, c, _ = PamgHIP.arrays(M)
    sort!(unique(Int64[x for x in c if x < lo || x >= hi]))
end

"Request exchange: every part tells each owner which of its rows it holds as ghosts."
function _build_plans(ghosts, offs)
    parts = linear_indices(ghosts)
    reqs = map(parts, ghosts) do p, g
        d = Dict{Int,Vector{Int64}}()
        for (q, id) in zip(_owner(g, offs), g)
            push!(get!(d, q, Int64[]), id)
        end
        d
    end
    got = _exchange(reqs, Int64)
    map(parts, ghosts, reqs, got) do p, g, rq, gt
        sends = Dict(q => ids .- offs[p] for (q, ids) in gt)
        nbrs = sort!(union(collect(keys(rq)), collect(keys(sends))))
        HostPlan(Int(offs[p+1] - offs[p]), Int(offs[p]), g, nbrs,
                 Int64[length(get(rq, q, Int64[])) for q in nbrs],
                 Int64[length(get(sends, q, Int64[])) for q in nbrs],
                 reduce(vcat, [get(sends, q, Int64[]) for q in nbrs]; init = Int64[]), sends)
    end
end

"Ghost rows of `mats` for every part's plan (the response half of the exchange)."
function _fetch_rows(plans, mats)
    rp_msgs = map((pl, M) -> Dict(q => PamgHIP.rows(M, idx .+ 1)[1] for (q, idx) in pl.sends), plans, mats)
    c_msgs = map((pl, M) -> Dict(q => Int64.(PamgHIP.rows(M, idx .+ 1)[2]) for (q, idx) in pl.sends), plans, mats)
    v_msgs = map((pl, M) -> Dict(q => PamgHIP.rows(M, idx .+ 1)[3] for (q, idx) in pl.sends), plans, mats)
    rps, cs, vs = _exchange(rp_msgs, Int64), _exchange(c_msgs, Int64), _exchange(v_msgs, Float64)
    map(plans, mats, rps, cs, vs) do pl, M, rp, c, v
        isempty(pl.ghost_ids) && return nothing
        rowptr, col, val = Int64[0], Int64[], Float64[]
        for q in sort!(collect(keys(rp)))                     # owners in ascending order = ghost order
            append!(rowptr, rp[q][2:end] .+ rowptr[end])
            append!(col, c[q]); append!(val, v[q])
        end
        length(rowptr) - 1 == length(pl.ghost_ids) || error("fetch_rows: ghost row count mismatch")
        HostCSR(rowptr, col, val, size(M)[2])
    end
end

"Local column ids (own first, then ghosts in ascending global order) of a global-column part."
function _localize(M::HostCSR, pl::Union{Nothing,HostPlan})
    rp, c, v = PamgHIP.arrays(M)
    pl === nothing && return (copy(rp), Int64.(c), copy(v), size(M)[2])
    lc = map(c) do x
        y = x - pl.col0
        0 <= y < pl.n_own ? Int64(y) : Int64(pl.n_own + searchsortedfirst(pl.ghost_ids, x) - 1)
    end
    (copy(rp), lc, copy(v), pl.n_own + length(pl.ghost_ids))
end

# tag = the plan's index-space identity, the same on every part (pamg_plan_set_tag; the
# hierarchy's plans: 1 + 3 (level - 1) + (A 0, P 1, R 2), as parallel_amg_amd/solver.py plan_tag)
function _device_plan(ctx, pl::HostPlan, tag::Integer = 0)
    isempty(pl.nbrs) && return nothing
    p = ExchangePlan(ctx, pl.n_own, length(pl.ghost_ids), Int32.(pl.nbrs .- 1), pl.recv_counts,
                     pl.send_counts, pl.send_idx .+ 1)
    tag != 0 && PamgHIP.set_tag!(p, tag)
    p
end

function _upload(ctx, M::HostCSR, pl::Union{Nothing,HostPlan}, tag::Integer = 0)
    rp, c, v, nc = _localize(M, pl)
    DeviceMatrix(ctx, rp, c, v, nc; plan = pl === nothing ? nothing : _device_plan(ctx, pl, tag), index_base = 0)
end
_plan_tag(l, op) = 1 + 3 * (l - 1) + (op === :A ? 0 : op === :P ? 1 : 2)

function _gather_full(mats, offs)
    rp_all = _allgather(map(M -> PamgHIP.arrays(M)[1], mats))
    c_all = _allgather(map(M -> Int64.(PamgHIP.arrays(M)[2]), mats))
    v_all = _allgather(map(M -> PamgHIP.arrays(M)[3], mats))
    map(rp_all, c_all, v_all) do rps, cs, vs
        rowptr, col, val = Int64[0], Int64[], Float64[]
        for k in 1:length(rps)
            append!(rowptr, rps[k][2:end] .+ rowptr[end]); append!(col, cs[k]); append!(val, vs[k])
        end
        HostCSR(rowptr, col, val, offs[end])
    end
end

"""
    HIPPVCycle(ctxs, A::PSparseMatrix; theta = 0.02, max_coarse = 1000, max_levels = 20,
               agglomerate = 32768, gpu_products = true, ncycles = 1)

Smoothed-aggregation hierarchy of A set up part by part (SPEC §S4; the driver of
parallel_amg_amd/hierarchy.py), levels ≥ 1 with ≤ `agglomerate` rows gathered whole on every
part (SPEC §S7), uploaded into one device VCycle per part. `ldiv!(x, M, b)` is one V-cycle.
A's rows must be a contiguous-block partition (uniform_partition / variable_partition).
"""
function HIPPVCycle(ctxs, A::PSparseMatrix; theta::Real = 0.02, max_coarse::Integer = 1000,
                    max_levels::Integer = 20, agglomerate::Integer = 32768, gpu_products::Bool = true,
                    ncycles::Integer = 1)
    rows = partition(axes(A, 1))
    nparts = length(rows)
    # replicated scalars / offsets are read with getany (the local part's copy under with_mpi)
    offs = Int64[0; cumsum(collect(getany(_allgather(map(ids -> Int64(own_length(ids)), rows)))))]
    # level 0 in global-column host CSR (0-based ids), per part
    Ah = map(own_own_values(A), own_ghost_values(A), partition(axes(A, 2))) do Aoo, Aog, cids
        cg = local_to_global(cids)
        ident = DeviceLayout(0, Int32[], Int32[], Int32.(cg), Int32[], Int64[])  # local id -> global id (1-based)
        rowptr, colv, valv = _own_rows_csr(Aoo, Aog, cids, ident)
        HostCSR(rowptr .- 1, colv .- 1, valv, offs[end])
    end
    levels = Dict{Symbol,Any}[]
    tail = nothing
    while true
        n = offs[end]
        if nparts > 1 && !isempty(levels) && 0 < agglomerate && n <= agglomerate
            full = _gather_full(Ah, offs)                         # the whole level on every part
            tail = map(ctxs, full) do ctx, F
                PamgHIP.setup_hierarchy(ctx, F; theta = theta, max_coarse = max_coarse,
                                        max_levels = max_levels - length(levels),
                                        gpu_products = gpu_products, reorder = :off)
            end
            break
        end
        parts = linear_indices(Ah)
        rho = _allreduce_max(map((M, p) -> PamgHIP.gershgorin(M, offs[p]), Ah, parts))
        omega = map(r -> 4.0 / (3.0 * r), rho)
        ghosts = map((M, p) -> nparts > 1 ? _ghost_ids(M, offs[p], offs[p+1]) : Int64[], Ah, parts)
        planA = _build_plans(ghosts, offs)
        lev = Dict{Symbol,Any}(:A => Ah, :offs => offs, :omega => omega, :planA => planA)
        push!(levels, lev)
        (n <= max_coarse || length(levels) >= max_levels) && break
        aggs = map((M, p) -> PamgHIP.aggregate(M, offs[p], theta), Ah, parts)
        coffs = Int64[0; cumsum(collect(getany(_allgather(map(a -> Int64(a[2]), aggs)))))]
        nc = coffs[end]
        (nc == 0 || nc >= n) && break
        T = map((a, p) -> PamgHIP.tentative(a[1], a[2], coffs[p], nc), aggs, parts)
        Tg = _fetch_rows(planA, T)
        ctx_or = gpu_products ? ctxs : map(_ -> nothing, ctxs)
        P = map(Ah, T, Tg, planA, parts, omega, ctx_or) do M, Tp, Tgp, pl, p, om, cx
            AT = PamgHIP.spgemm(M, offs[p], Tp, pl.ghost_ids, Tgp; ctx = cx)
            PamgHIP.smooth!(AT, M, offs[p], Tp, om)
        end
        Pg = _fetch_rows(planA, P)
        AP = map((M, Pp, Pgp, pl, p, cx) -> PamgHIP.spgemm(M, offs[p], Pp, pl.ghost_ids, Pgp; ctx = cx),
                 Ah, P, Pg, planA, parts, ctx_or)
        # R = P^T: each part transposes its rows per coarse owner and ships the pieces
        pieces = map(P, parts, ctx_or) do Pp, p, cx
            qs = nparts > 1 ? sort!(unique(_owner(unique(Int64.(PamgHIP.arrays(Pp)[2])), coffs))) : [p]
            Dict(q => PamgHIP.transpose_piece(Pp, offs[p], coffs[q], coffs[q+1]; ctx = cx) for q in qs)
        end
        prp = _exchange(map(d -> Dict(q => PamgHIP.arrays(M)[1] for (q, M) in d), pieces), Int64)
        pc = _exchange(map(d -> Dict(q => Int64.(PamgHIP.arrays(M)[2]) for (q, M) in d), pieces), Int64)
        pv = _exchange(map(d -> Dict(q => PamgHIP.arrays(M)[3] for (q, M) in d), pieces), Float64)
        R = map(parts, prp, pc, pv) do q, rp, c, v
            srcs = sort!(collect(keys(rp)))
            plist = [HostCSR(rp[p], c[p], v[p], n) for p in srcs]
            isempty(plist) ? HostCSR(zeros(Int64, coffs[q+1] - coffs[q] + 1), Int64[], Float64[], n) :
                length(plist) == 1 ? plist[1] : PamgHIP.hstack_rows(plist)
        end
        ghR = map((M, q) -> nparts > 1 ? _ghost_ids(M, offs[q], offs[q+1]) : Int64[], R, parts)
        planR = _build_plans(ghR, offs)
        APg = _fetch_rows(planR, AP)
        Ac = map((Rq, APq, APgq, pl, q, cx) -> PamgHIP.spgemm(Rq, offs[q], APq, pl.ghost_ids, APgq; ctx = cx),
                 R, AP, APg, planR, parts, ctx_or)
        ghP = map((M, p) -> nparts > 1 ? _ghost_ids(M, coffs[p], coffs[p+1]) : Int64[], P, parts)
        planP = _build_plans(ghP, coffs)
        merge!(lev, Dict(:P => P, :R => R, :planP => planP, :planR => planR, :coffs => coffs))
        Ah, offs = Ac, coffs
    end
    # upload: per level per part device matrices, then one VCycle per part (every per-part array
    # goes through map, so the same code runs under with_debug and with_mpi)
    L = length(levels)
    none = map(_ -> nothing, ctxs)
    dA = [map((c, M, pl) -> _upload(c, M, pl, _plan_tag(l, :A)), ctxs, levels[l][:A], levels[l][:planA]) for l in 1:L]
    withP = [l for l in 1:L if haskey(levels[l], :P)]
    dP = [map((c, M, pl) -> _upload(c, M, pl, _plan_tag(l, :P)), ctxs, levels[l][:P],
              (tail !== nothing && l == L) ? none : levels[l][:planP]) for l in withP]
    dR = [map((c, M, pl) -> _upload(c, M, pl, _plan_tag(l, :R)), ctxs, levels[l][:R], levels[l][:planR]) for l in withP]
    om = [lev[:omega] for lev in levels]
    if tail === nothing
        # coarsest level: every part assembles the whole matrix and the same inverse
        full = nparts == 1 ? levels[end][:A] : _gather_full(levels[end][:A], levels[end][:offs])
        ainv = map(PamgHIP.cholinv, full)
        rep, roffs = L - 1, levels[end][:offs]
    else
        ainv = map(Tv -> Tv.ainv, tail)
        rep, roffs = L, levels[end][:coffs]
    end
    nP = length(withP)
    hier = map(ctxs, tail === nothing ? none : tail, ainv, dA..., dP..., dR..., om...) do ctx, Tv, ai, rest...
        a = DeviceMatrix[rest[1:L]...]
        pm = DeviceMatrix[rest[L+1:L+nP]...]
        rm = DeviceMatrix[rest[L+nP+1:L+2nP]...]
        o = Float64[rest[L+2nP+1:end]...]
        if Tv !== nothing
            append!(a, Tv.A); append!(pm, Tv.P); append!(rm, Tv.R); append!(o, Tv.omega)
        end
        PamgHIP.VCycle(ctx, a, pm, rm, o, ai; rep_level = rep,
                       rep_offsets = nparts > 1 ? Vector{Int64}(roffs) : nothing, ncycles = ncycles)
    end
    HIPPVCycle(hier)
end

# The V-cycle preconditioner of a distributed hierarchy: one VCycle per part.
struct HIPPVCycle{A}
    parts::A
end
function LinearAlgebra.ldiv!(x::HIPPVector, M::HIPPVCycle, b::HIPPVector)
    w = _world(x.parts)
    if w === nothing
        foreach(ldiv!, x.parts, M.parts, b.parts)
    else  # one V-cycle from zero per ldiv! (the preconditioner), all parts in one call
        xs = collect(x.parts)
        foreach(v -> fill!(v, 0.0), xs)
        PamgHIP.world_vcycle!(w, xs, collect(M.parts), collect(b.parts); ncycles = first(collect(M.parts)).ncycles,
                               hist = false)
    end
    x
end

end # module

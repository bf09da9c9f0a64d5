% aiyagari_ge_multisection_gpu.m -- BASELINE config 4 from MATLAB/Octave (SURVEY §8(b) B2/B6).
%
% The GE search of Aiyagari_VFI.m:131-206 evaluated breadth-first: every midpoint the
% bisection could visit in its next `levels` steps (2^levels - 1 rates, each computed from its
% own bracket exactly as the sequential loop computes it) goes to the GPUs in ONE call,
% aiy_ge_batch_mex (VFI from the common warm start + Monte-Carlo supply with the uniforms block
% of the node's depth + K_d).  The script then walks the sequential loop's path through the
% evaluated tree, so r, r_history and the early stop are the bisection's.  Two rounds of
% levels = 6 (63 + 15 rates) cover the reference's 10 steps.
%
% Requires the gateways (see aiyagari_vfi_gpu.m).  n_devices = GPUs of this process.

clear; clc;
beta = 0.96; sigma = 5; alpha = 0.36; delta = 0.08; b = 0;
rho = 0.75; sigma_e = 0.75; N = 7; Na = 400;
tol = 1e-5; max_iter = 1000; T = 10000; n_steps = 10; levels = 6; n_devices = 1;

l_grid = ((1:N) - 4) * sigma_e;
edges = [-Inf, ((1:N-1) - 3.5) * sigma_e, Inf];
sd = sigma_e * sqrt(1 - rho^2);
P = zeros(N, N);
for i = 1:N
    for j = 1:N
        P(i, j) = integral(@(x) normpdf(x, rho * l_grid(i), sd), edges(j), edges(j + 1));
    end
end
s = exp(l_grid);
pi_stat = [P' - eye(N); ones(1, N)] \ [zeros(N, 1); 1];
labor = s * pi_stat;
kmax = delta^(1 / (alpha - 1));
amax = kmax^alpha + (1 - delta) * kmax;
a_grid = -b + (amax + b) * linspace(0, 1, Na).^2;
wage = @(r) (1 - alpha) * (alpha / (r + delta))^(alpha / (1 - alpha));

% the reference's stream: randi(N), randi(Na), then T-1 draws per simulation (initial + steps)
rng(5489, 'twister');
z1 = randi(N);
k1 = a_grid(randi(Na));
U = rand(T - 1, n_steps + 1);          % column d+1 = the draws of bisection step d

% common warm start: the r0 = 0.04 solution (every candidate starts from it)
[~, v0] = aiy_vfi_solve_mex(zeros(N, Na), a_grid, s, P, 0.04, wage(0.04), beta, sigma, tol, max_iter);

lo = -0.05; hi = 1 / beta - 1;
step = 0; done = false;
r_history = []; k_supply = []; k_demand = [];
tic;
while ~done && step < n_steps
    L = min(levels, n_steps - step);
    % breadth-first midpoints of the subtree below (lo, hi): node q has bracket br(q, :)
    br = [lo, hi]; nodes = zeros(0, 4);           % [r, lo, hi, depth]
    for lev = 1:L
        nb = zeros(0, 2);
        for q = 1:size(br, 1)
            m = (br(q, 1) + br(q, 2)) / 2;
            nodes(end + 1, :) = [m, br(q, 1), br(q, 2), step + lev]; %#ok<AGROW>
            nb = [nb; br(q, 1), m; m, br(q, 2)]; %#ok<AGROW>
        end
        br = nb;
    end
    [Ks, Kd, it] = aiy_ge_batch_mex(nodes(:, 1), v0, a_grid, s, P, alpha, delta, beta, sigma, ...
                                    labor, tol, max_iter, z1, k1, U(:, nodes(:, 4) + 1), n_devices);
    % walk the sequential loop's path (:196-204)
    for lev = 1:L
        q = find(nodes(:, 2) == lo & nodes(:, 3) == hi, 1);
        r = nodes(q, 1);
        r_history(end + 1) = r; k_supply(end + 1) = Ks(q); k_demand(end + 1) = Kd(q); %#ok<AGROW>
        if abs(Ks(q) - Kd(q)) < 1e-5
            done = true;
            break;
        elseif Ks(q) > Kd(q)
            hi = r;
        else
            lo = r;
        end
    end
    step = step + L;
end
fprintf('equilibrium r = %.10f (%d steps, %d candidate rates) in %.3f s\n', ...
        r_history(end), numel(r_history), size(nodes, 1), toc);

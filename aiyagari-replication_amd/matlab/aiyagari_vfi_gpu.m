% aiyagari_vfi_gpu.m -- host script for the MI355X solver (SURVEY.md §8(b) B6).
%
% The calibration, the general-equilibrium bisection and the reporting stay in MATLAB/Octave,
% as in the reference Aiyagari_VFI.m; the two inner loops it times are one gateway call each:
%   * the VFI loop (Aiyagari_VFI.m:65-90, GE copy :147-171)      -> aiy_vfi_solve_mex
%   * the Monte-Carlo capital supply (:94-129, GE copy :174-193) -> aiy_sim_capital_mex
% Build the gateways first (aiyagari-replication_amd/mex/Makefile header, or
%   mex -I../../include -L.. -laiyagari_hip <gateway>.c   /   mkoctfile --mex ...).
% Run from a fresh session: the uniforms below are MATLAB's stream from seed 5489, so the r
% trace is the reference's (tests/golden/a11_ge_vfi_defaults.npz holds it).

clear; clc;

% ---------------------------------------------------------------- calibration (:7-63)
beta = 0.96; sigma = 5; alpha = 0.36; delta = 0.08; b = 0;
rho = 0.75; sigma_e = 0.75; N = 7; Na = 400;
tol = 1e-5; max_iter = 1000; T = 10000;
use_step_gateways = false;   % true: keep the script's own VFI loop, one gateway call per sweep

% seven-state discretisation: grid points (i-4)*sigma_e, transition probabilities by
% integrating the conditional normal density over the fixed interval edges
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
A = [P' - eye(N); ones(1, N)];
pi_stat = A \ [zeros(N, 1); 1];
labor = s * pi_stat;

kmax = delta^(1 / (alpha - 1));
amax = kmax^alpha + (1 - delta) * kmax;
wmin = (1 - alpha) * (alpha / ((1 / beta - 1) + delta))^(alpha / (1 - alpha));
amin = min(b, wmin * s(1));           % the borrowing limit of Aiyagari_VFI.m:53-54
a_grid = amin + (amax - amin) * linspace(0, 1, Na).^2;

wage = @(r) (1 - alpha) * (alpha / (r + delta))^(alpha / (1 - alpha));
kdemand = @(r) labor * (alpha / (r + delta))^(1 / (1 - alpha));

% ---------------------------------------------------------------- initial solve at r = 0.04
rng(5489, 'twister');                 % the fresh-session stream the reference consumes
z1 = randi(N);
k1 = a_grid(randi(Na));
r = 0.04;
tic;
if use_step_gateways
    % the reference's loop (:65-90) with its sweep body (:68-83) swapped for the gateway
    v_old = zeros(N, Na);
    for iter = 1:max_iter
        [v_new, policy_k, policy_c, idx] = aiy_vfi_sweep_mex(v_old, a_grid, s, P, r, wage(r), ...
                                                             beta, sigma);
        if max(abs(v_new(:) - v_old(:))) < tol
            break;
        end
        v_old = v_new;
    end
else
    [v_new, v_old, policy_k, policy_c, iter] = ...
        aiy_vfi_solve_mex(zeros(N, Na), a_grid, s, P, r, wage(r), beta, sigma, tol, max_iter);
end
K_s = aiy_sim_capital_mex(policy_k, a_grid, P, z1, k1, rand(T - 1, 1), 1);
fprintf('r = %.4f: %d sweeps, K_s = %.6f\n', r, iter, K_s);

% ---------------------------------------------------------------- bisection on r (:131-206)
r_low = -0.05; r_high = 1 / beta - 1;
n_steps = 10;
r_history = zeros(n_steps, 1); k_supply = zeros(n_steps, 1); k_demand = zeros(n_steps, 1);
for step = 1:n_steps
    r = (r_low + r_high) / 2;
    % warm start from the previous solve's v_old (the reference's chained warm start)
    [v_new, v_old, policy_k, policy_c, iter, idx] = ...
        aiy_vfi_solve_mex(v_old, a_grid, s, P, r, wage(r), beta, sigma, tol, max_iter);
    [K_s, sim_k] = aiy_sim_capital_mex(policy_k, a_grid, P, z1, k1, rand(T - 1, 1), 1);
    K_d = kdemand(r);
    r_history(step) = r; k_supply(step) = K_s; k_demand(step) = K_d;
    fprintf('step %2d: r = %.6f, K_s = %.6f, K_d = %.6f (%d sweeps)\n', step, r, K_s, K_d, iter);
    if abs(K_s - K_d) < 1e-5
        break;
    elseif K_s > K_d
        r_high = r;
    else
        r_low = r;
    end
end
fprintf('equilibrium r = %.10f after %.3f s\n', r, toc);

% ---------------------------------------------------------------- stationary histogram (A10)
% the on-grid policy's fixed point on the (z, a) grid: a deterministic alternative to the
% Monte-Carlo mean (new; the reference has no histogram update).  idx is the last solve's
% 1-based argmax, returned by the gateway (policy_k == a_grid(idx)).
[lambda, K_hist] = aiy_dist_stationary_mex(idx, a_grid, P, ones(N, Na) / (N * Na), 1e-12, ...
                                           10000, 1);
fprintf('histogram K = %.6f, Monte-Carlo K = %.6f\n', K_hist, K_s);

% krusell_smith_vfi_gpu.m -- host script for the Krusell-Smith solver (SURVEY §8(b) B6).
%
% Mirrors the outer loop of Krusell_Smith_VFI.m:138-296 with its hot sections as gateway calls:
%   * the VFI for the current ALM coefficients (:143-204)  -> ks_vfi_solve_mex
%       (policy improvement by fminbnd every 5th iteration, 50 Jacobi Howard sweeps; the
%        n_devices argument shards the aggregate-capital slices over the GPUs of this process)
%   * the shock panel (:57-94)                            -> ks_shocks_mex (once)
%   * the panel simulation (:206-248)                     -> ks_simulate_capital_mex
% The regression of log K' on log K per aggregate state and the damped update of B stay here.
% params = [beta alpha delta k_min k_max ug ub l_bar mu z_grid(1) z_grid(2) eps_grid(1) eps_grid(2)].

clear; clc;
beta = 0.99; alpha = 0.36; delta = 0.025; k_min = 0.0001; k_max = 1000;
ug = 0.04; ub = 0.10; mu = 0; l_bar = 1 / (1 - ub);
z_grid = [1.01, 0.99]; eps_grid = [1, 0];
k_size = 100; K_size = 4; T = 1100; population = 10000; T_discard = 100;
howard_steps = 50; tol_vfi = 1e-6; max_vfi = 10000; tol_B = 1e-6; max_B = 100;
update_B = 0.3; n_devices = 1;
use_step_gateways = false;   % true: keep the script's own VFI loop (:143-204) around the steps
params = [beta alpha delta k_min k_max ug ub l_bar mu z_grid eps_grid];

k_grid = linspace(0, 1, k_size).^7 * (k_max - k_min) + k_min;
k_grid(1) = k_min; k_grid(end) = k_max;
K_grid = linspace(30, 50, K_size);

% 4 x 4 transition over s = (z, eps): aggregate durations 8 / 8 quarters, unemployment
% durations 1.5 (good) and 2.5 (bad), spells 25 % longer / shorter across regime switches
pgg = 1 - 1 / 8; pbb = 1 - 1 / 8; pgb = 1 - pgg; pbg = 1 - pbb;
p00 = [1 - 1 / 1.5, 1 - 1 / 2.5];            % stay unemployed: good, bad
p00_gb = 1.25 * p00(2); p00_bg = 0.75 * p00(1);
p10 = @(u0, u1, p) (u1 - u0 * p) / (1 - u0);  % employed -> unemployed, given u' and p00
q00 = [p00(1), p00_gb; p00_bg, p00(2)];        % [from g: to g, to b; from b: to g, to b]
zt = [pgg, pgb; pbg, pbb];
u = [ug, ub];
P = zeros(4, 4);
for zi = 1:2
    for zj = 1:2
        q = q00(zi, zj);
        e2u = p10(u(zi), u(zj), q);
        % rows/cols in the script's order (g,e), (b,e), (g,u), (b,u)
        P(zi, zj) = zt(zi, zj) * (1 - e2u);       % employed -> employed
        P(zi, zj + 2) = zt(zi, zj) * e2u;          % employed -> unemployed
        P(zi + 2, zj) = zt(zi, zj) * (1 - q);      % unemployed -> employed
        P(zi + 2, zj + 2) = zt(zi, zj) * q;        % unemployed -> unemployed
    end
end

% shock panel from the fresh-session stream (draw order of :57-94)
rng(5489, 'twister');
n_draws = (T - 1) + population + (T - 1) * population;
[zi_shock, epsi_shock] = ks_shocks_mex(T, population, rand(n_draws, 1), params);

k_opt = 0.9 * repmat(k_grid', [1, K_size, 4]);
value = log(0.1 / 0.9 * k_opt) / (1 - beta);
k_population = ones(population, 1) * K_grid(1);
B = [0, 1, 0, 1];
for B_iter = 1:max_B
    tic;
    if use_step_gateways
        % the reference's loop with its improvement (:148-168) and Howard sweeps (:172-192)
        % swapped for the step gateways; the relative-difference stop (:195-203) stays here
        for vfi_iter = 1:max_vfi
            value_old = value;
            if mod(vfi_iter - 1, 5) == 0
                k_opt = ks_policy_improve_mex(value, k_grid, K_grid, B, P, params);
            end
            value = ks_howard_mex(value, k_opt, k_grid, K_grid, B, P, params, howard_steps);
            rel = abs(value(:) - value_old(:)) ./ (abs(value_old(:)) + 1e-10);
            if max(rel) < tol_vfi
                break;
            end
        end
    else
        [value, k_opt, vfi_iter] = ks_vfi_solve_mex(value, k_opt, k_grid, K_grid, B, P, ...
                                                    params, howard_steps, tol_vfi, max_vfi, ...
                                                    n_devices);
    end
    [K_ts, k_population] = ks_simulate_capital_mex(k_opt, k_grid, K_grid, zi_shock, ...
                                                   epsi_shock, k_population);
    % OLS of log K(t+1) on [1, log K(t)] per aggregate state (t >= T_discard)
    t = (T_discard:T - 1)';
    good = zi_shock(t) == 0;
    B_new = zeros(1, 4);
    for g = [1, 0]
        sel = t(good == g);
        X = [ones(numel(sel), 1), log(K_ts(sel))];
        Y = log(K_ts(sel + 1));
        if ~isempty(sel)
            B_new(3 - 2 * g:4 - 2 * g) = (X \ Y)';
        end
    end
    diff_B = max(abs(B_new - B));
    fprintf('ALM %3d: %d VFI iterations, B_new = [%.4f %.4f %.4f %.4f], diff %.2e (%.2f s)\n', ...
            B_iter, vfi_iter, B_new, diff_B, toc);
    if diff_B < tol_B
        break;
    end
    B = update_B * B_new + (1 - update_B) * B;
end
